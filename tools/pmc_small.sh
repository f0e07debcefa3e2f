#!/bin/bash
# rocprofv3 counter passes over a small bench run (each pass its own run; no tracing domains)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $ctrs | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --stats -d $R/gpurun_out/pmc/$tag -o run -- python3 $R/bench.py --docs ${DOCS:-20000} --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc/$tag.log 2>&1
done
