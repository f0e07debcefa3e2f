#!/bin/bash
# One GPU call: GPU tests (TESTS, default all), then the default bench (BENCH_ARGS) and, optionally,
# extra bench workloads (EXTRA="cfg3 cfg5"), each under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bench
mkdir -p $O
cd $R
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 700 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for w in ${EXTRA:-}; do
  timeout -k 10 600 python -u bench.py --workload $w --no-cpu-baseline --steps 3 > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $O/bench_$w.log; exit 1; }
  tail -1 $O/bench_$w.log
done
