#!/bin/bash
# Round-2 PMC passes of the bench workload (one rocprofv3 --pmc pass per counter group, each under its
# own kill timeout; MI355X_MICROARCH.md "rocprofv3 PMC slots": <= 8 SQ, <= 4 TCC per pass, FETCH_SIZE
# and WRITE_SIZE in separate passes).  WORKLOAD=cfg2|cfg5, DOCS as bench.py --docs.
# Writes gpurun_out/pmc_<workload>/pmc_summary.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
W=${WORKLOAD:-cfg2}
O=$R/gpurun_out/pmc_$W
mkdir -p $O
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  echo "pass $i: $ctrs"
  timeout -k 10 -s KILL ${PASS_TIMEOUT:-170} rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $O/p$i -o run -- \
    python3 $R/bench.py --workload $W ${DOCS:+--docs $DOCS} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $O/p$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done <<LIST
FETCH_SIZE
WRITE_SIZE
${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH
TCC_HIT_sum TCC_MISS_sum}
LIST
PMC_WORKLOAD="$(grep '^{"metric"' $O/p1.log | head -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["workload"])')" \
  python3 $R/tools/pmc_summary.py $O > $O/pmc_summary.json && cat $O/pmc_summary.json
