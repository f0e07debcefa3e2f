#!/bin/bash
# streamed batch timeline with load / upload traces
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04w}
mkdir -p $O
cd $R
for c in ${CHUNKS:-262144 1000000}; do
  GG_STREAM_TRACE=1 GG_LOAD_TRACE=1 timeout -k 10 300 python -u tools/stream_probe.py 1000000 $c > $O/probe_$c.log 2>&1 || { tail -20 $O/probe_$c.log; exit 1; }
  grep -E "evals/s" $O/probe_$c.log
done
