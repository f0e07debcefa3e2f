"""Diagnostic: lane-group (split walk) results against one lane per tile, rule by rule (tf plans)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import synth  # noqa: E402

CASES = {
    "list": "rule r { planned_values.root_module.resources[*].values.bucket == 'x' }",
    "flist": "rule r { planned_values.root_module.resources[ type == 'aws_s3_bucket' ].values.bucket == 'x' }",
    "let": "let b = planned_values.root_module.resources[ type == 'aws_s3_bucket' ]\nrule r { %b.values.bucket == 'x' }",
    "letcount": "let b = planned_values.root_module.resources[ type == 'aws_s3_bucket' ]\nrule r { %b !empty }",
    "map": "rule r { planned_values.root_module.resources[0].values.* == 'x' }",
}


def run(text, docs, env):
    for k in ("GG_LANE_GROUP", "GG_SPLIT_WALK"):
        os.environ.pop(k, None)
    os.environ.update(env)
    s = guard_amd.Session()
    s.add_rules(text, "p.guard")
    s.add_docs(docs, ["g-%d.json" % i for i in range(len(docs))])
    s.eval(1)
    out = json.loads(s.report()[0])
    s.close()
    return out


docs = synth.tf_corpus(2, start=300, n_resources=20)
for name, text in CASES.items():
    a = run(text, docs, {"GG_LANE_GROUP": "1"})
    for g in ("2", "4"):
        b = run(text, docs, {"GG_LANE_GROUP": g})
        na = [len(json.dumps(d)) for d in a]
        nb = [len(json.dumps(d)) for d in b]
        print(name, "G=" + g, "same" if a == b else "DIFF", na, nb)
        if a != b and g == "2":
            print(json.dumps(b[0], indent=1)[:3000])
