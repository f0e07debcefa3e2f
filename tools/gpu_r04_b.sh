#!/bin/bash
# Round 4: GPU suite (JSON reports now rendered on the device by default) + the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r04b}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
TAG=$T bash tools/gpu_tests.sh || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
cut -c1-600 $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['e2e']))"
