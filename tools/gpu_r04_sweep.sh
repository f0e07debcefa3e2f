#!/bin/bash
# lane-kernel launch knobs on one box: waves per CU of the lane grid, direct-record chunk
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04sweep}
mkdir -p $O
cd $R
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 5 ${BENCH_ARGS:-} > $O/$tag.json 2> $O/$tag.log || { echo "$tag failed"; tail -3 $O/$tag.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['detail']['kernel_ms_mean'], d['value'])"
}
run base GG_NONE=1 && run chunk48 GG_REC_CHUNK=48 && run chunk64 GG_REC_CHUNK=64 && run chunk96 GG_REC_CHUNK=96 && run chunk128 GG_REC_CHUNK=128 && \
run chunk64b GG_REC_CHUNK=64 && run base2 GG_NONE=1
