#!/bin/bash
# device reporter check: its parity tests, then the default bench line (e2e with the device reporter)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r04c}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_report.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['e2e']))"
