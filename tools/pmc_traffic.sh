#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the evaluation kernels on the bench workload (one pass per counter).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc
mkdir -p $O
for ctr in FETCH_SIZE WRITE_SIZE ${EXTRA_PMC:-}; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$ctr -o run -- \
    python3 $R/bench.py --docs ${DOCS:-1000000} --steps 1 --warmup 1 --no-cpu-baseline > $O/$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -5 $O/$ctr.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/pmc"
for f in sorted(glob.glob(O + "/*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"][:48], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        if "gg::" in k:
            print("%-48s %-12s per-dispatch %.4g (n=%d)" % (k, c, sum(v) / len(v), len(v)))
PY
