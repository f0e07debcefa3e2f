#!/bin/bash
# streamed batch entry: its tests, then the default bench line with e2e_stream
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04s}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['e2e'])[:200]); print(json.dumps(d.get('e2e_stream')))"
