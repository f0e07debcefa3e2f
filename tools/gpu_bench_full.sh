#!/bin/bash
# One GPU call: the default bench line (what the driver runs), optionally after the GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-benchfull}
mkdir -p $O
cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.log | cut -c1-3000
tail -5 $O/bench.err
