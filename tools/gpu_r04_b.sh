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
timeout -k 10 500 python -u bench.py --workload cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_cfg4.json 2> $O/bench_cfg4.log || { echo "cfg4 failed"; tail -5 $O/bench_cfg4.log; exit 1; }
cut -c1-800 $O/bench_cfg4.json
