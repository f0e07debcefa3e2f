#!/bin/bash
# the whole GPU suite, then smoke and the default bench line (the driver's round-end sequence)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04full}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TAG=${TAG:-r04full} bash tools/gpu_r04_final.sh
