#!/bin/bash
# device allocation cache: stream tests, the streamed timeline, then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04t}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_device_report.py -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -2 $O/pytest.log
GG_LOAD_TRACE=1 timeout -k 10 300 python -u tools/stream_probe.py 1000000 262144 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -E "evals/s|returned" $O/probe.log
timeout -k 10 900 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['e2e'])[:300]); print(json.dumps(d.get('e2e_stream')))"
