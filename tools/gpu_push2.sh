#!/bin/bash
# streamed entry with the shader copy-out (default for streams): CU-mask variants of render / copy
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-push2}; mkdir -p $O; cd $R
for c in 0 16 32; do
  echo "[push2] $(date +%T) stream probe GG_PUSH_CUS=$c"
  GG_PUSH_CUS=$c timeout -k 10 240 python3 -u tools/stream_probe.py 1000000 262144 native > $O/stream_cus$c.log 2>&1 || { tail -20 $O/stream_cus$c.log; exit 1; }
  tail -1 $O/stream_cus$c.log
done
echo "[push2] $(date +%T) stream probe copy engine (GG_D2H_PUSH=0)"
GG_D2H_PUSH=0 timeout -k 10 240 python3 -u tools/stream_probe.py 1000000 262144 native > $O/stream_sdma.log 2>&1 || { tail -20 $O/stream_sdma.log; exit 1; }
tail -1 $O/stream_sdma.log
echo "[push2] done"
