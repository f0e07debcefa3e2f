#!/bin/bash
# D2H rate vs device-memory churn (tools/d2h_frag.py), then the report A/B with the pinned staging's NUMA trace
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-frag}; mkdir -p $O; cd $R
echo "[frag] $(date +%T) d2h"
timeout -k 10 240 python3 -u tools/d2h_frag.py > $O/d2h_frag.log 2>&1 || { tail -20 $O/d2h_frag.log; exit 1; }
cat $O/d2h_frag.log
echo "[frag] $(date +%T) report_ab"
GG_PINNED_TRACE=1 timeout -k 10 300 python3 -u tools/report_ab.py 262144 > $O/report_ab.log 2> $O/report_ab.err || { tail -20 $O/report_ab.err; exit 1; }
cat $O/report_ab.log; grep pinned $O/report_ab.err | sort | uniq -c
echo "[frag] done"
