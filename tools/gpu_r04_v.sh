#!/bin/bash
# streamed batch at several chunk sizes (timeline)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04v}
mkdir -p $O
cd $R
for c in 1000000 500000 131072; do
  GG_STREAM_TRACE=1 GG_DREPORT_TRACE=1 timeout -k 10 300 python -u tools/stream_probe.py 1000000 $c > $O/probe_$c.log 2>&1 || { tail -20 $O/probe_$c.log; exit 1; }
  grep -E "evals/s" $O/probe_$c.log
done
