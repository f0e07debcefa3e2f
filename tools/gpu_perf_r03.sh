#!/bin/bash
# One GPU call (round 3 diagnostics): cfg2 + cfg5 bench lines (no CPU baseline / e2e) and the stats
# build's per-file counters + cycle breakdown for cfg5 and cfg2.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-perf}
mkdir -p $O
cd $R
echo "bench cfg2"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > $O/bench_cfg2.log 2>&1 || { echo "bench cfg2 failed"; tail -20 $O/bench_cfg2.log; exit 1; }
grep '^{"metric"' $O/bench_cfg2.log | cut -c1-400
echo "bench cfg5"
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline --no-e2e > $O/bench_cfg5.log 2>&1 || { echo "bench cfg5 failed"; tail -20 $O/bench_cfg5.log; exit 1; }
grep '^{"metric"' $O/bench_cfg5.log | cut -c1-400
if [ -n "${STATS:-}" ]; then
for P in cfg5 cfg2; do
  echo "stats $P"
  GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_stats.so PACK=$P timeout -k 10 300 python -u tools/kernel_stats.py ${DOCS:-20000} > $O/kernel_stats_$P.json 2> $O/kernel_stats_$P.err || { echo "kernel_stats failed"; tail -20 $O/kernel_stats_$P.err; exit 1; }
done
fi
echo done
