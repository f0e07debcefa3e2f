#!/bin/bash
# One GPU call: the -m gpu suite (one process), then smoke.  Output under gpurun_out/$TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-tests}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
