#!/bin/bash
# Round 4: GPU suite + smoke, direct-record A/B on cfg2, cfg4 lane vs wave, the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r04a}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
TAG=$T bash tools/gpu_tests.sh || exit 1
for ch in 0 32; do
  GG_REC_CHUNK=$ch timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e \
    > $O/bench_cfg2_chunk$ch.json 2> $O/bench_cfg2_chunk$ch.log || { echo "cfg2 chunk $ch failed"; tail -5 $O/bench_cfg2_chunk$ch.log; exit 1; }
  cut -c1-700 $O/bench_cfg2_chunk$ch.json
done
for m in lane wave; do
  timeout -k 10 400 python -u bench.py --workload cfg4 --docs ${CFG4_DOCS:-2048} --mode $m --steps 3 --warmup 1 \
    --no-cpu-baseline --no-e2e > $O/bench_cfg4_$m.json 2> $O/bench_cfg4_$m.log || { echo "cfg4 $m failed"; tail -5 $O/bench_cfg4_$m.log; exit 1; }
  cut -c1-700 $O/bench_cfg4_$m.json
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
cut -c1-2500 $O/bench.json
