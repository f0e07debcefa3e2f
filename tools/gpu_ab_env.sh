#!/bin/bash
# Kernel-only bench lines of one workload under alternating environment settings (A/B on one box).
#   WORKLOAD=cfg4 SETTINGS="GG_SIZE_ORDER=0 GG_SIZE_ORDER=1" ROUNDS=2 bash tools/gpu_ab_env.sh
# A setting "-" runs with no extra variable.  Lines under gpurun_out/$TAG/ab_<workload>_<k>_<setting>.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
W=${WORKLOAD:-cfg4}
cd $R
for k in $(seq 1 ${ROUNDS:-2}); do
  for s in $SETTINGS; do
    f=$O/ab_${W}_${k}_${s//=/_}.json
    if [ "$s" = "-" ]; then
      timeout -k 10 300 python3 -u bench.py --workload $W --steps ${STEPS_N:-3} --warmup 1 --no-e2e --no-cpu-baseline > $f 2> $f.log || { tail -5 $f.log; exit 1; }
    else
      env $s timeout -k 10 300 python3 -u bench.py --workload $W --steps ${STEPS_N:-3} --warmup 1 --no-e2e --no-cpu-baseline > $f 2> $f.log || { tail -5 $f.log; exit 1; }
    fi
    python3 -c "import json; d=json.load(open('$f')); print('$W $k $s', d['value'], d['ms_per_step'])"
  done
done
