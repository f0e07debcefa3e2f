#!/bin/bash
# cfg4 lane-group size sweep (kernel only): G = auto, 4, 8, 32, 64
set -o pipefail
O=gpurun_out/${TAG:-sweep}; mkdir -p $O
B="python -u bench.py --workload cfg4 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline"
for g in auto 4 8 32 64; do
  if [ $g = auto ]; then timeout -k 10 240 $B > $O/g_$g.json 2> $O/g_$g.err || exit 1
  else GG_LANE_GROUP=$g timeout -k 10 240 $B > $O/g_$g.json 2> $O/g_$g.err || exit 1; fi
  python -c "import json; d=json.load(open('$O/g_$g.json')); print('G=$g', d['value'], d['ms_per_step'], d['detail']['lane_tiles_retried_in_wave_mode'])"
done
