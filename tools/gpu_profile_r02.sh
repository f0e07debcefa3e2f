#!/bin/bash
# One GPU call: rocprofv3 kernel-trace summary of the bench command, a 2-rank rehearsal of the
# multi-GPU bench path on ONE GPU (gloo tallies, both ranks pinned to device 0; never N=8), and the
# cfg5 PMC passes (LDS-staged regex DFA tables: LDS bank conflicts next to HBM traffic).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "kernel trace"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/trace.log 2>&1 || { echo "trace failed"; tail -20 $O/trace.log; exit 1; }
grep '^{"metric"' $O/trace.log | tail -1 | cut -c1-400
cd $R
echo "2-rank rehearsal"
GG_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --docs 100000 --dist-backend gloo --no-cpu-baseline --no-e2e > $O/bench2.log 2>&1 || { echo "2-rank bench failed"; tail -30 $O/bench2.log; exit 1; }
grep '^{' $O/bench2.log | tail -1 | cut -c1-300
echo "cfg5 pmc"
WORKLOAD=cfg5 PASSES="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
  bash $R/tools/pmc_r02.sh > $O/pmc_cfg5.log 2>&1 || { echo "cfg5 pmc failed"; tail -20 $O/pmc_cfg5.log; exit 1; }
tail -3 $O/pmc_cfg5.log
