#!/bin/bash
# A/B of the product library against libcfnguard_mi355x_ab.so on one box: WORKLOADS (default cfg2), alternating
set -o pipefail
O=gpurun_out/${TAG:-ab}; mkdir -p $O
B="python -u bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline"
for w in ${WORKLOADS:-cfg2}; do
for v in prod ab prod ab; do
  L=cloudformation-guard_amd/libcfnguard_mi355x.so; [ $v = ab ] && L=cloudformation-guard_amd/libcfnguard_mi355x_ab.so
  GG_LIB=$L timeout -k 10 300 $B --workload $w > $O/${w}_$v.json 2> $O/${w}_$v.err || exit 1
  python -c "import json; d=json.load(open('$O/${w}_$v.json')); print('$w $v', d['value'], d['ms_per_step'])"
done
done
