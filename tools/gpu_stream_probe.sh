#!/bin/bash
# the streamed JSON leg (bench e2e_stream) standalone, one child process per run; RUNS="name[:VAR=v[,VAR=v]]" ...
# with the per-chunk timeline (GG_STREAM_TRACE) on stderr
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-stream_probe}
mkdir -p $O
cd $R
for run in ${RUNS:-a b}; do
  name=${run%%:*}; envs=""; [ "$run" != "$name" ] && envs=${run#*:}
  env GG_STREAM_TRACE=1 ${envs//,/ } timeout -k 10 300 python3 -u tools/stream_leg.py cfg2 0 ${DOCS:-1000000} 50 json 262144 0 16 \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  echo "$name $(tail -1 $O/$name.json)"
done
