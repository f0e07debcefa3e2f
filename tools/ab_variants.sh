#!/bin/bash
# A/B of build variants on the cfg-2 bench: VARIANTS="g5 g6" runs the product library, then each
# libcfnguard_mi355x_<v>.so (built beforehand with `python cloudformation-guard_amd/build.py <v>`).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abv
mkdir -p $O
cd $R
for v in base ${VARIANTS}; do
  if [ $v = base ]; then lib=$R/cloudformation-guard_amd/libcfnguard_mi355x.so; else lib=$R/cloudformation-guard_amd/libcfnguard_mi355x_$v.so; fi
  GG_LIB=$lib timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 1; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'kernel_ms', d['detail']['kernel_ms_mean'], 'value', d['value'], 'tiles', d['detail']['tiles_fail_pass_skip_err'], 'recs', d['detail']['record_bytes'], 'tally', d['detail']['rule_tallies_sum'])"
done
