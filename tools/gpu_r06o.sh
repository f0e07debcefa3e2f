#!/bin/bash
# cfg2: quick-walk A/B; cfg4: lane-group size and heap-budget sweep
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline"
for v in prod ab prod ab; do
  L=cloudformation-guard_amd/libcfnguard_mi355x.so; [ $v = ab ] && L=cloudformation-guard_amd/libcfnguard_mi355x_ab.so
  GG_LIB=$L timeout -k 10 300 $B --workload cfg2 > $O/cfg2_$v.json 2> $O/cfg2_$v.err || exit 1
  python -c "import json; d=json.load(open('$O/cfg2_$v.json')); print('cfg2 $v', d['value'], d['ms_per_step'])"
done
for cfg in "16 48" "8 48" "32 48" "16 64" "32 128"; do
  set -- $cfg
  GG_LANE_GROUP=$1 GG_GROUP_HEAP_GB=$2 timeout -k 10 300 $B --workload cfg4 > $O/cfg4_$1_$2.json 2> $O/cfg4_$1_$2.err || exit 1
  python -c "import json; d=json.load(open('$O/cfg4_$1_$2.json')); print('cfg4 G=$1 heap=$2', d['value'], d['ms_per_step'], d['detail'].get('lane_tiles_retried_in_wave_mode'))"
done
