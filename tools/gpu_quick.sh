#!/bin/bash
# One GPU call: selected GPU tests (TESTS, default all -m gpu), then an optional bench (BENCH_ARGS).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/quick
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 400 python -u bench.py $BENCH_ARGS > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log
fi
