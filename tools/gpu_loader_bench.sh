#!/bin/bash
# One GPU call: bench with the device JSON loader, plus its rocprofv3 kernel-trace summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/loader
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --loader device --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --loader device --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
