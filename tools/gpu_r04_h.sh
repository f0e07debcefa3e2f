#!/bin/bash
# cfg4 (few large Terraform plans): lane vs wave kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04h}
mkdir -p $O
cd $R
for m in lane wave; do
  timeout -k 10 600 python -u bench.py --workload cfg4 --mode $m --no-cpu-baseline --no-e2e --steps 3 > $O/cfg4_$m.json 2> $O/cfg4_$m.log || { echo "bench $m failed"; tail -5 $O/cfg4_$m.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg4_$m.json')); print('$m', d['value'], d['ms_per_step'], d['detail'].get('lane_tiles_retried_in_wave_mode'))"
done
