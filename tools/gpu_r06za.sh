#!/bin/bash
# size-ordered lane-group batches (cfg4 A/B) and the windowed YAML scans (loader tests + rate)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06za
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_yaml.py tests/test_gpu_loader.py tests/test_gpu_lane_groups.py -x -q \
  --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --format yaml --steps 1 --warmup 0 --no-e2e --no-cpu-baseline > $O/yaml.json 2> $O/yaml.log || { tail -5 $O/yaml.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/yaml.json')); print('yaml loader', d['detail']['device_loader'])"
TAG=r06za WORKLOAD=cfg4 SETTINGS="GG_SIZE_ORDER=0 GG_SIZE_ORDER=1" ROUNDS=2 bash tools/gpu_ab_env.sh
