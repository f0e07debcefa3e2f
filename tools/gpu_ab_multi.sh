#!/bin/bash
# kernel ms per launch of each library in $VARIANTS on each workload in $WORKLOADS (bench.py, no CPU baseline / e2e)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG}; mkdir -p $O; cd $R
for w in ${WORKLOADS:-cfg2}; do
  for v in $VARIANTS; do
    L=$R/cloudformation-guard_amd/libcfnguard_mi355x_$v.so; [ "$v" = main ] && L=$R/cloudformation-guard_amd/libcfnguard_mi355x.so
    GG_LIB=$L timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline --no-e2e --steps 3 > $O/bench_${w}_$v.json 2> $O/bench_${w}_$v.log || { tail -5 $O/bench_${w}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/bench_${w}_$v.json')); print('$w $v', d['ms_per_step'], d['detail']['kernel_ms_mean'], d['detail']['lane_tiles_retried_in_wave_mode'])"
  done
done
