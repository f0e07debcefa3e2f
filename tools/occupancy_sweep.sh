#!/bin/bash
# Rebuilds the lane kernel at several occupancy targets and times the cfg-2 workload (diagnostic).
set -e
R=$GRAFT_REPO_ROOT
cd $R
D=${DOCS:-200000}
for w in ${WAVES:-2 4 8}; do
  rm -f cloudformation-guard_amd/build/eval_kernel.o
  GG_LANE_WAVES_PER_EU=$w python -c "import __graft_entry__ as g; g.build()" > gpurun_out/sweep_build_$w.log 2>&1
  for per_cu in $(( w * 4 )) $(( w * 2 )); do
    GG_LANE_WAVES_PER_CU=$per_cu timeout -k 10 300 python bench.py --docs $D --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_${w}_${per_cu}.log 2>&1
    echo "eu=$w percu=$per_cu $(tail -n 1 gpurun_out/sweep_${w}_${per_cu}.log | cut -c1-200)"
  done
done
