#!/bin/bash
# Console reporter GPU tests, then the stats-build per-function call counts (cfg5, cfg2).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/console
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_console.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -40; }
bash tools/gpu_stats_only.sh || exit 1
exit $rc
