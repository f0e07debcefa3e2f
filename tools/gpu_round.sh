#!/bin/bash
# One GPU session: the steps named in $STEPS, in order, each under its own time limit; the first failing
# step ends the session (no GPU work after a failure).  Steps:
#   tests          python -m pytest tests -m gpu ($PYTEST_K selects)
#   smoke          __graft_entry__.smoke()
#   bench:<cfg>    bench.py --workload <cfg> $BENCH_ARGS (the full line: cpu_baseline, e2e)
#   ktrace:<cfg>   rocprofv3 --kernel-trace --stats of bench.py --workload <cfg> (5 timed steps)
#   pmc:<cfg>      FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh)
#   lds:<cfg>      SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE / SQ_INSTS_LDS pass
#   ldsnfa         the same counters over the NFA rule pack (tools/nfa_probe.py)
# Outputs under gpurun_out/$TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-run}
mkdir -p $O
export TMPDIR=/tmp
docs_of() { case $1 in cfg4) echo 8192;; cfg5) echo 303031;; *) echo 1000000;; esac; }
for step in $STEPS; do
  W=${step#*:}
  echo "[gpu_round] $(date +%T) $step"
  case $step in
    tests)
      (cd $R && timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
         ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1) || { tail -40 $O/pytest.log; exit 1; }
      tail -3 $O/pytest.log;;
    smoke)
      (cd $R && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1) || { tail -20 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log;;
    bench:*)
      (cd $R && timeout -k 10 900 python3 -u bench.py --workload $W $BENCH_ARGS > $O/bench_$W.json 2> $O/bench_$W.log) || { tail -10 $O/bench_$W.log; exit 1; }
      cut -c1-2500 $O/bench_$W.json;;
    ktrace:*)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_$W -o run -- \
         python3 $R/bench.py --workload $W --docs $(docs_of $W) --steps 5 --warmup 1 --no-cpu-baseline --no-e2e \
         > $O/ktrace_$W.log 2>&1) || { tail -8 $O/ktrace_$W.log; exit 1; }
      grep '^{"metric"' $O/ktrace_$W.log | cut -c1-400
      head -6 $O/ktrace_$W/run_kernel_stats.csv 2>/dev/null || find $O/ktrace_$W -name "*kernel_stats.csv" -exec head -6 {} \; ;;
    pmc:*)
      WORKLOAD=$W DOCS=$(docs_of $W) bash $R/tools/pmc_traffic.sh > $O/pmc_$W.log 2>&1 || { tail -8 $O/pmc_$W.log; exit 1; }
      cp $R/gpurun_out/pmc_$W/pmc_summary.json $O/pmc_$W.json
      grep hbm_bytes $O/pmc_$W.json;;
    lds:*)
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace \
         --output-format csv -d $O/lds_$W -o run -- python3 $R/bench.py --workload $W --docs $(docs_of $W) --steps 1 \
         --warmup 1 --no-cpu-baseline --no-e2e > $O/lds_$W.log 2>&1) || { tail -8 $O/lds_$W.log; exit 1; }
      echo "lds $W done";;
    ldsnfa)
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace \
         --output-format csv -d $O/lds_nfa -o run -- python3 $R/tools/nfa_probe.py 200000 > $O/lds_nfa.log 2>&1) || { tail -8 $O/lds_nfa.log; exit 1; }
      echo "lds nfa done";;
    *) echo "unknown step $step"; exit 2;;
  esac
done
echo "[gpu_round] $(date +%T) done"
