#!/bin/bash
# A/B of evaluator builds under rocprofv3 --pmc (diagnostic): for each library in LIBS (suffixes of
# cloudformation-guard_amd/libcfnguard_mi355x<suffix>.so, "" = product), one pass per counter group
# on the bench workload; prints per-dispatch means of the lane kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcab
mkdir -p $O
D=${DOCS:-200000}
for v in ${LIBS:-"" _prev}; do
  lib=$R/cloudformation-guard_amd/libcfnguard_mi355x$v.so
  i=0
  for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
              "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH"; do
    i=$((i+1))
    GG_LIB=$lib timeout -k 10 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $O/v$v-$i -o run -- \
      python3 $R/bench.py --docs $D --steps 1 --warmup 1 --no-cpu-baseline > $O/v$v-$i.log 2>&1 || { echo "pmc $v $ctrs failed"; tail -5 $O/v$v-$i.log; exit 1; }
  done
  python3 - "$O" "v$v" <<'PY'
import csv, glob, collections, sys
O, tag = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(O + "/" + tag + "-*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "guard_eval_lanes_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(tag, " ".join("%s=%.4g" % (k, sum(v) / len(v)) for k, v in sorted(agg.items())))
PY
done
