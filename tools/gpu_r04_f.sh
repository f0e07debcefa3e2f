#!/bin/bash
# device YAML loader: its parity / refusal tests and the loader suite
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04f}
mkdir -p $O
cd $R
GG_LOAD_DIAG=1 timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_yaml.py tests/test_gpu_loader.py} -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -60
exit $rc
