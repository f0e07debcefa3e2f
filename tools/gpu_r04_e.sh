#!/bin/bash
# e2e phase timeline: device loader phases (GG_LOAD_TRACE) and the device reporter's render / copy-out overlap
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r04e}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_device_report.py tests/test_gpu_parity.py tests/test_gpu_loader.py} -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
fi
GG_LOAD_TRACE=1 GG_DREPORT_TRACE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 2 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep "\[load\]\|\[upload\]\|\[bench" $O/bench.log | head -40
grep dreport $O/bench.log | tail -6
if [ -n "$ALSO_HOST_ARENA" ]; then
GG_RESIDENT_ARENA=0 GG_LOAD_TRACE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 2 > $O/bench_h.json 2> $O/bench_h.log || { echo "bench (host arena) failed"; tail -5 $O/bench_h.log; exit 1; }
grep "\[upload\]\|upload (" $O/bench_h.log
python3 -c "import json; d=json.load(open('$O/bench_h.json')); print('host arena', d['value'], json.dumps(d['e2e'])[:300])"
fi
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['e2e']))"
