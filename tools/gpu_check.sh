#!/bin/bash
# One GPU call: parity tests, smoke, short bench, rocprofv3 kernel-trace summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
find $O/prof -name "*stats*" | head
