#!/bin/bash
# device loader: GPU loader tests, then the cfg2 bench with the device loader (kernel GB/s of text)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-loader_ab}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_loader.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --loader device --no-cpu-baseline --no-e2e --steps 2 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['detail']['device_loader'])"
