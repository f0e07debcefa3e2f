#!/bin/bash
# Occupancy A/B on the cfg-2 bench (diagnostic): RUNS="lib:waves_per_cu ..." (lib "" = product).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abocc
mkdir -p $O
cd $R
for run in ${RUNS:-":8"}; do
  v=${run%%:*}; w=${run##*:}
  lib=$R/cloudformation-guard_amd/libcfnguard_mi355x${v}.so
  GG_LIB=$lib GG_LANE_WAVES_PER_CU=$w timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > $O/bench${v}_$w.log 2>&1 || { echo "bench $run failed"; tail -20 $O/bench${v}_$w.log; exit 1; }
  tail -1 $O/bench${v}_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$run', 'kernel_ms', d['detail']['kernel_ms_mean'], 'value', d['value'], 'tiles', d['detail']['tiles_fail_pass_skip_err'], 'recs', d['detail']['record_bytes'])"
done
