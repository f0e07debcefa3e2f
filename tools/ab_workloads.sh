#!/bin/bash
# A/B of the product library against libcfnguard_mi355x_<v>.so on several workloads (kernel only),
# after the GPU parity tests named by $TESTS (default: parity + workloads).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-abw}
mkdir -p $O
cd $R
if [ "${TESTS:-x}" != none ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_workloads.py} -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for w in ${WORKLOADS:-cfg2 cfg5 cfg3}; do
  for v in base ${VARIANTS:-ab}; do
    if [ $v = base ]; then lib=$R/cloudformation-guard_amd/libcfnguard_mi355x.so; else lib=$R/cloudformation-guard_amd/libcfnguard_mi355x_$v.so; fi
    GG_LIB=$lib timeout -k 10 300 python -u bench.py --workload $w --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_${w}_$v.log 2>&1 || { echo "bench $w $v failed"; tail -20 $O/bench_${w}_$v.log; exit 1; }
    grep '^{"metric"' $O/bench_${w}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w $v', 'kernel_ms', d['detail']['kernel_ms_mean'], 'value', d['value'], 'frac', d['roofline']['frac'], 'tiles', d['detail']['tiles_fail_pass_skip_err'], 'recs', d['detail']['record_bytes'])"
  done
done
