#!/bin/bash
# session vs streamed report copy-out in one process (tools/report_ab.py), then the streamed probe
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-rab}; mkdir -p $O; cd $R
echo "[rab] $(date +%T) report_ab"
GG_DREPORT_TRACE=1 timeout -k 10 300 python3 -u tools/report_ab.py 262144 > $O/report_ab.log 2> $O/report_ab.err || { tail -20 $O/report_ab.err; exit 1; }
cat $O/report_ab.log
echo "[rab] $(date +%T) stream probe"
GG_STREAM_TRACE=1 timeout -k 10 240 python3 -u tools/stream_probe.py 1000000 262144 native > $O/stream.log 2>&1 || { tail -20 $O/stream.log; exit 1; }
tail -1 $O/stream.log
echo "[rab] done"
