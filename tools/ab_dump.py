"""Diagnostic: dump validate_structured output per (rules file, document) for the library GG_LIB
names, so two builds can be diffed (tools/ab_dump.py OUT.json PACK NDOCS)."""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "cloudformation-guard_amd")]
import guard_amd  # noqa: E402
import synth  # noqa: E402

out_path, pack, ndocs = sys.argv[1], sys.argv[2], int(sys.argv[3])
G = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", pack)
rules = [(f, open(os.path.join(G, f)).read()) for f in sorted(os.listdir(G)) if f.endswith(".guard")]
docs = synth.cfn_corpus(ndocs, start=500, n_resources=12)
res = {}
for name, text in rules:
    for i, d in enumerate(docs):
        try:
            out, code = guard_amd.validate_structured([(name, text)], [("doc%d.json" % i, d)])
            res["%s|%d" % (name, i)] = out
        except guard_amd.GuardError as e:
            res["%s|%d" % (name, i)] = "ERR %s" % e.message
json.dump({"docs": docs, "res": res}, open(out_path, "w"))
print("dumped", len(res))
