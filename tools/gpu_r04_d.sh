#!/bin/bash
# NFA-regex parity on the device, then the device reporter's render / copy-out timeline (GG_DREPORT_TRACE)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r04d}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GG_DREPORT_TRACE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 2 > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep dreport $O/bench.log | tail -40
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['e2e']))"
