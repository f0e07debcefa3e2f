#!/bin/bash
# cfg3 (22 files): direct-record chunk under the reservation cap (16) vs 32 / 64
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04sweep3}
mkdir -p $O
cd $R
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-e2e --steps 3 > $O/$tag.json 2> $O/$tag.log || { echo "$tag failed"; tail -3 $O/$tag.log; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['detail']['kernel_ms_mean'], d['value'])"
}
run c16 GG_REC_CHUNK=16 && run c32 GG_REC_CHUNK=32 && run c8 GG_REC_CHUNK=8 && run c16b GG_REC_CHUNK=16
