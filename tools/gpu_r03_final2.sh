#!/bin/bash
# Round-3 closing pass: full GPU suite + smoke, the default bench line, kernel-trace statistics, and
# FETCH_SIZE / WRITE_SIZE passes for cfg2, cfg5 and cfg3.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r03z} bash tools/gpu_tests.sh || exit 1
O=$R/gpurun_out/${TAG:-r03z}
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-300
TAG=${TAG:-r03z}prof bash tools/gpu_r03_prof.sh || exit 1
WORKLOAD=cfg3 PMC_WORKLOAD="cfg3: 1000000 synthetic CFN templates/GPU (50 resources) x 22-file rule pack" \
  bash tools/pmc_traffic.sh > $O/pmc_cfg3.log 2>&1 || { echo "pmc cfg3 failed"; tail -5 $O/pmc_cfg3.log; exit 1; }
grep hbm_bytes $O/pmc_cfg3.log
