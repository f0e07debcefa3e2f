#!/bin/bash
# Round 3 bench lines: cfg2 with the device loader (e2e), cfg5 and cfg3 (kernel only).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r03lines}
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --loader device --no-cpu-baseline > $O/bench_dev.log 2>&1 || { echo "bench device failed"; tail -20 $O/bench_dev.log; exit 1; }
grep '^{"metric"' $O/bench_dev.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline --no-e2e > $O/bench_cfg5.log 2>&1 || { echo "bench cfg5 failed"; tail -20 $O/bench_cfg5.log; exit 1; }
grep '^{"metric"' $O/bench_cfg5.log | cut -c1-300
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-e2e > $O/bench_cfg3.log 2>&1 || { echo "bench cfg3 failed"; tail -20 $O/bench_cfg3.log; exit 1; }
grep '^{"metric"' $O/bench_cfg3.log | cut -c1-300
