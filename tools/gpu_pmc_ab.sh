#!/bin/bash
# FETCH_SIZE / WRITE_SIZE and instruction counters of the cfg2 lane kernel for each library in $LIBS
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-pmcab}; mkdir -p $O
export TMPDIR=/tmp
for v in $LIBS; do
  mkdir -p $O/$v
  for ctr in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU+SQ_INSTS_SALU+SQ_INSTS_LDS+SQ_INSTS_VMEM_RD+SQ_INSTS_VMEM_WR+SQ_WAVE_CYCLES+SQ_BUSY_CYCLES; do
    (cd /tmp && GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_$v.so timeout -k 10 300 rocprofv3 --pmc ${ctr//+/ } --kernel-trace --output-format csv \
      -d $O/$v/$ctr -o run -- python3 $R/bench.py --workload ${WORKLOAD:-cfg2} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e \
      > $O/$v/$ctr.log 2>&1) || { echo "pmc $v $ctr failed"; tail -5 $O/$v/$ctr.log; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $O/$v > $O/pmc_$v.json && python3 -c "
import json; d=json.load(open('$O/pmc_$v.json')); l=d['kernels']['lanes']
print('$v hbm', d['hbm_bytes_per_launch'], 'fetch_kib', l['fetch_kib_raw'], 'write_kib', l['write_kib_raw'], l['counters_mean_per_dispatch'])"
done
