#!/bin/bash
# One GPU call: GPU parity suite (writes gpurun_out/ffi_latency.json), then the cfg3 and cfg5 bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wl
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in cfg3 cfg5; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $O/bench_$w.log; exit 1; }
  grep '^{"metric"' $O/bench_$w.log | tail -1 | cut -c1-260
done
