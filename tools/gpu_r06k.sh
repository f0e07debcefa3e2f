#!/bin/bash
# parked chunks: lane-group parity, variant latencies, cfg4 kernel line
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lane_groups.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
GSIZES=16 EXTRA=tools/cfg4_variants2.guard SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/variants2.jsonl 2> $O/variants2.err || exit 1
SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/solo.jsonl 2> $O/solo.err || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --workload cfg4 > $O/cfg4.json 2> $O/cfg4.err || exit 1
python -c "import json; d=json.load(open('$O/cfg4.json')); print('cfg4', d['value'], d['ms_per_step'], d['detail'].get('lane_tiles_retried_in_wave_mode'))"
