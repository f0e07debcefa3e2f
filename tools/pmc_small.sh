#!/bin/bash
# rocprofv3 passes over the bench workload: one kernel-trace/stats pass, then one run per PMC
# group (counters never share a run with tracing domains).  Output: $R/gpurun_out/prof/<tag>/
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=${DOCS:-1000000}
mkdir -p $R/gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/trace -o run -- \
  python3 $R/bench.py --docs $D --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof/trace.log 2>&1
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM"; do
  tag=$(echo $ctrs | cut -d' ' -f1)
  timeout -k 10 400 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $R/gpurun_out/prof/$tag -o run -- \
    python3 $R/bench.py --docs $D --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof/$tag.log 2>&1
done
