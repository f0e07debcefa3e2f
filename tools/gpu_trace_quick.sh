#!/bin/bash
# Kernel-trace summary of a short cfg-2 bench (diagnostic): per-kernel average durations.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_${TAG:-q}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
cut -d, -f1-4 "$f" | head -8
