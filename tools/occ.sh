#!/bin/bash
# occupancy experiment over prebuilt variants (python cloudformation-guard_amd/build.py eu<N>)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/occ
for cfg in ${CFGS:-":8" "eu3:12" "eu4:16"}; do
  v=${cfg%%:*}; w=${cfg##*:}
  lib=$R/cloudformation-guard_amd/libcfnguard_mi355x${v:+_$v}.so
  GG_LIB=$lib GG_LANE_WAVES_PER_CU=$w timeout -k 10 200 python bench.py --docs 1000000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/occ/$v-$w.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/occ/$v-$w.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/occ/$v-$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["detail"]["kernel_ms_mean"], d["value"], d["detail"]["tiles_fail_pass_skip_err"])')"
done
