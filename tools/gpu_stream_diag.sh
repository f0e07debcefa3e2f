#!/bin/bash
# Streamed-entry timeline diagnostics (GPU): per-chunk and per-block render / copy spans of
# cfn_guard_validate_batch_stream on 1M cfg2 texts, chunk-size and copy-engine variants.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-sdiag}; mkdir -p $O; cd $R
run() {  # name, env..., -- args
  local name=$1; shift
  echo "[sdiag] $(date +%T) $name"
  env "$@" timeout -k 10 240 python3 -u tools/stream_probe.py $ARGS > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  tail -1 $O/$name.log
}
ARGS="1000000 262144" run trace GG_STREAM_TRACE=1 GG_DREPORT_TRACE=1
ARGS="1000000 1000000" run one_chunk GG_STREAM_TRACE=1
ARGS="1000000 262144" run nosdma HSA_ENABLE_SDMA=0 GG_STREAM_TRACE=1
ARGS="1000000 262144" run block128k GG_DREPORT_BLOCK=131072 GG_STREAM_TRACE=1
# lane-kernel residency sweep (scratch + heap working set against latency hiding)
for W in 8 12 16; do
  echo "[sdiag] $(date +%T) waves/CU $W"
  GG_LANE_WAVES_PER_CU=$W timeout -k 10 300 python3 -u bench.py --workload cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
    > $O/waves_$W.json 2> $O/waves_$W.log || { tail -10 $O/waves_$W.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('waves', sys.argv[2], d['ms_per_step'], d['detail']['kernel_ms_mean'])" $O/waves_$W.json $W
done
echo "[sdiag] done"
