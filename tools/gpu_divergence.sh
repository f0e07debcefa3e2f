#!/bin/bash
# Divergence A/B (diagnostic): per-file lane-kernel cost on the cfg-2 corpus, on identical documents
# (GG_SYNTH_MOD=1) and on documents grouped 64 to a resource-type sequence (GG_SYNTH_SHAPE_GROUP=64).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/div
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/bench_files.py 200000 > $O/base.json 2>$O/base.err || { echo base failed; tail $O/base.err; exit 1; }
GG_SYNTH_MOD=1 timeout -k 10 200 python -u tools/bench_files.py 200000 > $O/same.json 2>$O/same.err || { echo same failed; tail $O/same.err; exit 1; }
GG_SYNTH_SHAPE_GROUP=64 timeout -k 10 200 python -u tools/bench_files.py 200000 > $O/grp64.json 2>$O/grp64.err || { echo grp failed; tail $O/grp64.err; exit 1; }
python3 - <<'PY'
import json
d={k:json.load(open("gpurun_out/div/%s.json"%k)) for k in ("base","same","grp64")}
for f in d["base"]:
    print("%-48s" % f, " ".join("%s %7.3f ms %9d rec" % (k, d[k][f]["kernel_ms"], d[k][f]["records"]) for k in d))
print("total", {k: round(sum(v["kernel_ms"] for v in d[k].values()), 2) for k in d})
PY
