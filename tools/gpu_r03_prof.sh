#!/bin/bash
# Kernel-trace statistics of the default bench (cfg2) and FETCH_SIZE / WRITE_SIZE passes for cfg2 and cfg5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r03prof}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/ktrace.log 2>&1 || { echo "kernel trace failed"; tail -5 $O/ktrace.log; exit 1; }
grep '^{"metric"' $O/ktrace.log | cut -c1-400
WORKLOAD=cfg2 PMC_WORKLOAD="cfg2: 1000000 synthetic CFN templates/GPU (50 resources) x 7-file rule pack" \
  bash $R/tools/pmc_traffic.sh > $O/pmc_cfg2.log 2>&1 || { echo "pmc cfg2 failed"; tail -5 $O/pmc_cfg2.log; exit 1; }
grep hbm_bytes $O/pmc_cfg2.log
WORKLOAD=cfg5 PMC_WORKLOAD="cfg5: 303031 AWS Config snapshots/GPU (9999863 configuration items) x 2-file network-reachability pack" \
  DOCS=303031 bash $R/tools/pmc_traffic.sh > $O/pmc_cfg5.log 2>&1 || { echo "pmc cfg5 failed"; tail -5 $O/pmc_cfg5.log; exit 1; }
grep hbm_bytes $O/pmc_cfg5.log
