#!/bin/bash
# Diagnostic PMC passes (one rocprofv3 --pmc run per line of $PASSES, each under its own kill timeout;
# per-pass block limits: MI355X_MICROARCH.md "rocprofv3 PMC slots").  Writes gpurun_out/$TAG/pmc_summary.json
# (mean per dispatch of every counter, per kernel).  WORKLOAD / DOCS / BENCH_EXTRA as bench.py options.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
W=${WORKLOAD:-cfg2}
O=$R/gpurun_out/${TAG:-pmc_diag}
mkdir -p $O
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  echo "pass $i: $ctrs"
  timeout -k 10 -s KILL ${PASS_TIMEOUT:-150} rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $O/p$i -o run -- \
    python3 $R/bench.py --workload $W ${DOCS:+--docs $DOCS} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e ${BENCH_EXTRA:-} > $O/p$i.log 2>&1 \
    || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done <<< "$PASSES"
python3 - "$O" > $O/pmc_summary.json <<'PY'
import collections, csv, glob, json, os, sys
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("gg::", "")
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: {c: sum(v) / len(v) for c, v in sorted(d.items())} for k, d in per.items()
                  if "lanes" in k or "resource_type" in k}, indent=1))
PY
cat $O/pmc_summary.json
