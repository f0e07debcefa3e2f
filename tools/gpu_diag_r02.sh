#!/bin/bash
# One GPU call (diagnostic): GPU tests, then per-rules-file evaluator counters + cycle breakdown
# (stats build) and per-file kernel times (product build) on the cfg-2 corpus.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${DIAG_DIR:-diag}
mkdir -p $O
cd $R
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_stats.so PACK=${PACK:-cfg2} timeout -k 10 300 python -u tools/kernel_stats.py ${DOCS:-100000} > $O/kernel_stats.json 2> $O/kernel_stats.err || { echo "kernel_stats failed"; tail -20 $O/kernel_stats.err; exit 1; }
if [ "${PACK:-cfg2}" = micro ]; then
  timeout -k 10 300 python -u tools/micro.py ${DOCS:-100000} > $O/bench_files.json 2> $O/bench_files.err || { echo "micro failed"; tail -20 $O/bench_files.err; exit 1; }
else
  timeout -k 10 300 python -u tools/bench_files.py ${DOCS:-100000} > $O/bench_files.json 2> $O/bench_files.err || { echo "bench_files failed"; tail -20 $O/bench_files.err; exit 1; }
fi
echo done
