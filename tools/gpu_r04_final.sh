#!/bin/bash
# the driver's round-end sequence on one GPU: smoke, then the default bench line (CPU baseline included)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r04final}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -8 $O/bench.log; exit 1; }
cat $O/bench.json | cut -c1-3000
