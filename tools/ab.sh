#!/bin/bash
# Quick GPU iteration: parity tests, then the cfg-2 bench without the CPU baseline.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'kernel_ms', d['detail']['kernel_ms_mean'], 'frac', d['roofline']['frac'], 'tiles', d['detail']['tiles_fail_pass_skip_err'], 'recs', d['detail']['record_bytes'])"
