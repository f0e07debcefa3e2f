#!/bin/bash
# quick filters: the new parity test, the whole -m gpu suite + smoke, then cfg4 / cfg2 kernel lines
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_quick_filters.py > $O/quick.log 2>&1 || { tail -40 $O/quick.log; exit 1; }
tail -1 $O/quick.log
TAG=r06l bash tools/gpu_tests.sh || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline"
timeout -k 10 300 $B --workload cfg4 > $O/cfg4.json 2> $O/cfg4.err || exit 1
python -c "import json; d=json.load(open('$O/cfg4.json')); print('cfg4', d['value'], d['ms_per_step'], d['detail'].get('lane_tiles_retried_in_wave_mode'))"
timeout -k 10 400 $B --workload cfg2 > $O/cfg2.json 2> $O/cfg2.err || exit 1
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2', d['value'], d['ms_per_step'])"
SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/solo.jsonl 2> $O/solo.err
