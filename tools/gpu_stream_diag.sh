#!/bin/bash
# Streamed-entry diagnostics (GPU): cfn_guard_validate_batch_stream on 1M cfg2 texts with the Python
# per-piece callback against the library's native counter (gg_count_write), chunked and as one chunk;
# per-chunk / per-block render and copy spans with STREAM_TRACE=1.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-sdiag}; mkdir -p $O; cd $R
run() {  # name, env...
  local name=$1; shift
  echo "[sdiag] $(date +%T) $name"
  env "$@" timeout -k 10 240 python3 -u tools/stream_probe.py $ARGS > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  tail -1 $O/$name.log
}
if [ -n "$STREAM_TRACE" ]; then TR="GG_STREAM_TRACE=1 GG_DREPORT_TRACE=1"; else TR="GG_STREAM_TRACE=1"; fi
ARGS="1000000 262144 native" run native_262k $TR
ARGS="1000000 262144 py" run py_262k $TR
ARGS="1000000 1000000 native" run native_1m $TR
echo "[sdiag] done"
