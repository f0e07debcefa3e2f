#!/bin/bash
# Round 4, first call: GPU suite + smoke, cfg4 lane vs wave (small), the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04a}
mkdir -p $O
cd $R
TAG=${TAG:-r04a} bash tools/gpu_tests.sh || exit 1
for m in lane wave; do
  timeout -k 10 400 python -u bench.py --workload cfg4 --docs ${CFG4_DOCS:-2048} --mode $m --steps 3 --warmup 1 \
    --no-cpu-baseline --no-e2e > $O/bench_cfg4_$m.json 2> $O/bench_cfg4_$m.log || { echo "cfg4 $m failed"; tail -5 $O/bench_cfg4_$m.log; exit 1; }
  cut -c1-600 $O/bench_cfg4_$m.json
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
cut -c1-1500 $O/bench.json
