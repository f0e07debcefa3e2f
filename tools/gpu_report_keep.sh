#!/bin/bash
# report copy-out A/B across sessions: default, render buffers kept with the buffer set, smaller report blocks
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-rkeep}; mkdir -p $O; cd $R
for v in default keep block16k; do
  case $v in default) E="";; keep) E="GG_KEEP_RENDER=1";; block16k) E="GG_DREPORT_BLOCK=16384";; esac
  echo "[rkeep] $(date +%T) $v"
  env $E timeout -k 10 300 python3 -u tools/report_ab.py 262144 > $O/report_ab_$v.log 2> $O/report_ab_$v.err || { tail -20 $O/report_ab_$v.err; exit 1; }
  cat $O/report_ab_$v.log
done
echo "[rkeep] done"
