#!/bin/bash
# Round 3 checkpoint: full GPU suite + smoke, then the default bench line (cfg2, CPU baseline, e2e).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r03chk} bash tools/gpu_tests.sh || exit 1
O=$R/gpurun_out/${TAG:-r03chk}
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-600
