#!/bin/bash
# One GPU call (round 2, final build): default bench line, bench with the device JSON loader (e2e),
# rocprofv3 kernel-trace summary, and the cfg-2 PMC passes (HBM bytes + SQ + TCP/L2 latency counters).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${FINAL_TAG:-final2}
mkdir -p $O
cd $R
echo "bench"
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | tail -1 | cut -c1-300
echo "bench device loader"
timeout -k 10 400 python -u bench.py --loader device --steps 3 --no-cpu-baseline > $O/bench_devload.log 2>&1 || { echo "bench devload failed"; tail -20 $O/bench_devload.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
echo "kernel trace"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
grep '^{"metric"' $O/trace.log | tail -1 | cut -c1-200
echo "pmc"
PASSES="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum
TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE" \
  PASS_TIMEOUT=170 bash $R/tools/pmc_r02.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
cp -r $R/gpurun_out/pmc_cfg2 $O/ 2>/dev/null
echo done
