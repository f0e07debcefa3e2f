#!/bin/bash
# cfg4 group-size / heap sweep under the size order; per-pass kernel times of the device YAML loader
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zb
mkdir -p $O
cd $R
TAG=r06zb WORKLOAD=cfg4 SETTINGS="- GG_LANE_GROUP=8 GG_LANE_GROUP=32 GG_GROUP_HEAP_GB=64" ROUNDS=1 bash tools/gpu_ab_env.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/yprof -o run -- \
  python3 $R/bench.py --format yaml --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/yprof.log 2>&1 || { tail -5 $O/yprof.log; exit 1; }
find $O/yprof -name "*kernel_stats.csv" -exec head -14 {} \; | cut -d, -f1-5
