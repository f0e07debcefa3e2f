#!/bin/bash
# YAML: loader tests, then the cfg2 bench over block-style YAML templates (device YAML loader)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04g}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_yaml.py -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GG_LOAD_TRACE=1 timeout -k 10 600 python -u bench.py --format yaml --no-cpu-baseline --steps 3 > $O/bench_yaml.json 2> $O/bench_yaml.log || { echo "bench failed"; tail -8 $O/bench_yaml.log; exit 1; }
grep "\[load\]\|\[bench" $O/bench_yaml.log | head -30
python3 -c "import json; d=json.load(open('$O/bench_yaml.json')); print(d['value'], d['config']['workload']); print(json.dumps(d['e2e'])[:400]); print(json.dumps(d['detail'].get('device_loader')))"
