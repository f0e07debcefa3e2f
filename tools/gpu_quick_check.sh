#!/bin/bash
# a change's quick GPU check: lane-group / quick-filter / workload parity, then the cfg4 kernel line and
# the one-plan rule latencies.  TAG names the output directory.
set -o pipefail
O=gpurun_out/${TAG:-qc}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lane_groups.py tests/test_gpu_quick_filters.py tests/test_gpu_workloads.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --workload cfg4 > $O/cfg4.json 2> $O/cfg4.err || exit 1
python -c "import json; d=json.load(open('$O/cfg4.json')); print('cfg4', d['value'], d['ms_per_step'], d['detail'].get('lane_tiles_retried_in_wave_mode'))"
SIZE=2000 PACK=cfg4 timeout -k 10 200 python -u tools/rule_split_timing.py 1 > $O/solo.jsonl 2> $O/solo.err
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --workload cfg2 > $O/cfg2.json 2> $O/cfg2.err || exit 1
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --workload cfg5 > $O/cfg5.json 2> $O/cfg5.err || exit 1
python -c "import json; d=json.load(open('$O/cfg5.json')); print('cfg5', d['value'], d['ms_per_step'])"
