#!/bin/bash
# Round-3 checkpoint: full GPU suite + smoke, the default bench line (cfg2, CPU baseline, e2e), the
# device-loader bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r03fin} bash tools/gpu_tests.sh || exit 1
O=$R/gpurun_out/${TAG:-r03fin}
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-400
timeout -k 10 400 python -u bench.py --loader device --no-cpu-baseline > $O/bench_dev.log 2>&1 || { echo "bench device failed"; tail -20 $O/bench_dev.log; exit 1; }
grep '^{"metric"' $O/bench_dev.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dev e2e', d['e2e']['value'], d['detail']['device_loader'])"
