#!/bin/bash
# Kernel-only bench lines alternating the product library and the A/B build (libcfnguard_mi355x_ab.so) on one
# box, then the parity tests on the A/B build.  WORKLOADS="cfg2 cfg5" ROUNDS=2 PYTEST_FILES="tests/..."
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-lib_ab}
mkdir -p $O
cd $R
for k in $(seq 1 ${ROUNDS:-2}); do
  for w in ${WORKLOADS:-cfg2}; do
    for v in prod ab; do
      L=$R/cloudformation-guard_amd/libcfnguard_mi355x.so; [ $v = ab ] && L=$R/cloudformation-guard_amd/libcfnguard_mi355x_ab.so
      GG_LIB=$L timeout -k 10 300 python3 -u bench.py --workload $w --steps 5 --warmup 1 --no-e2e --no-cpu-baseline \
        > $O/${w}_${v}_$k.json 2> $O/${w}_${v}_$k.log || { tail -5 $O/${w}_${v}_$k.log; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${w}_${v}_$k.json')); print('$w $v $k', d['value'], d['ms_per_step'])"
    done
  done
done
if [ -n "$PYTEST_FILES" ]; then
  GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_ab.so timeout -k 10 600 python -u -m pytest $PYTEST_FILES -x -q \
    --timeout 240 --timeout-method thread > $O/pytest_ab.log 2>&1 || { tail -20 $O/pytest_ab.log; exit 1; }
  tail -2 $O/pytest_ab.log
fi
