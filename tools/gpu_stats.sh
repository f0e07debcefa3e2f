#!/bin/bash
# One GPU call: GPU parity suite, then per-file evaluator counters of the stats build (tools/kernel_stats.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stats
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GG_LIB=$R/cloudformation-guard_amd/libcfnguard_mi355x_stats.so timeout -k 10 300 python -u tools/kernel_stats.py ${STATS_DOCS:-100000} > $O/kernel_stats.json 2> $O/kernel_stats.err || { echo stats failed; tail $O/kernel_stats.err; exit 1; }
cat $O/kernel_stats.json
