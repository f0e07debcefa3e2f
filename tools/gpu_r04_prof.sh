#!/bin/bash
# Round 4 profiles: kernel-trace statistics of the default bench (cfg2), then FETCH_SIZE / WRITE_SIZE
# passes (one counter per pass, MI355X_MICROARCH.md) for cfg2, cfg3, cfg4 and cfg5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04prof}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/ktrace.log 2>&1 || { echo "kernel trace failed"; tail -5 $O/ktrace.log; exit 1; }
grep '^{"metric"' $O/ktrace.log | cut -c1-300
for W in ${WORKLOADS:-cfg2 cfg3 cfg5 cfg4}; do
  case $W in
    cfg2) D=1000000; PW="cfg2: 1000000 synthetic CFN templates/GPU (50 resources) x 7-file rule pack";;
    cfg3) D=1000000; PW="cfg3: 1000000 synthetic CFN templates/GPU (50 resources) x 22-file rule pack";;
    cfg5) D=303031; PW="cfg5: 303031 AWS Config snapshots/GPU (9999863 configuration items) x 2-file network-reachability pack";;
    cfg4) D=8192; PW="cfg4: 8192 Terraform plans/GPU (9021401 resource_changes, 200-2000 per plan) x 2-file terraform pack";;
  esac
  WORKLOAD=$W DOCS=$D PMC_WORKLOAD="$PW" bash $R/tools/pmc_traffic.sh > $O/pmc_$W.log 2>&1 || { echo "pmc $W failed"; tail -5 $O/pmc_$W.log; exit 1; }
  cp $R/gpurun_out/pmc_$W/pmc_summary.json $O/pmc_$W.json
  grep hbm_bytes $O/pmc_$W.log
done
