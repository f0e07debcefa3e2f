#!/bin/bash
# full bench lines (cfg2 default, cfg4) with the report cross-check; YAML loader rate after the comment scan
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zc
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --format yaml --steps 1 --warmup 0 --no-e2e --no-cpu-baseline > $O/yaml.json 2> $O/yaml.log || { tail -5 $O/yaml.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/yaml.json')); print('yaml loader', d['detail']['device_loader']['text_GBps'], d['detail']['device_loader']['kernel_ms'])"
TAG=r06zc STEPS="bench:cfg2 bench:cfg4" bash tools/gpu_round.sh
