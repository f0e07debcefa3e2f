#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the evaluation kernels on the bench workload, one rocprofv3 --pmc pass
# per counter (MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Writes gpurun_out/pmc/pmc_summary.json; copy it to profiles/pmc_r01.json so bench.py reports
# roofline.traffic from it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_${WORKLOAD:-cfg2}
mkdir -p $O
# a pass may hold several counters joined by '+' (EXTRA_PMC="SQ_INSTS_VALU+SQ_INSTS_SALU")
for ctr in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC:-}; do
  timeout -k 10 300 rocprofv3 --pmc ${ctr//+/ } --kernel-trace --output-format csv -d $O/$ctr -o run -- \
    python3 $R/bench.py --docs ${DOCS:-1000000} --workload ${WORKLOAD:-cfg2} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $O/$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $O/$ctr.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O > $O/pmc_summary.json && cat $O/pmc_summary.json
