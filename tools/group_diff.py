"""Diagnostic: the first document whose lane-group report differs from the one-lane report (tf pack)."""
import difflib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import rulepack  # noqa: E402
import synth  # noqa: E402


def run(rules, docs, env):
    for k in ("GG_LANE_GROUP", "GG_SPLIT_WALK"):
        os.environ.pop(k, None)
    os.environ.update(env)
    s = guard_amd.Session()
    for n, t in rules:
        s.add_rules(t, n)
    s.add_docs(docs, ["g-%d.json" % i for i in range(len(docs))])
    s.eval(1)
    out = s.report()[0]
    s.close()
    return json.loads(out)


rules = rulepack.rule_pack(sys.argv[1] if len(sys.argv) > 1 else "cfg4")
docs = synth.tf_corpus(9, start=300, n_resources=150)
base = run(rules, docs, {"GG_LANE_GROUP": "1"})
for env in ({"GG_LANE_GROUP": "2", "GG_SPLIT_WALK": "0"}, {"GG_LANE_GROUP": "2"}, {"GG_LANE_GROUP": "16"}):
    got = run(rules, docs, env)
    bad = [i for i in range(len(docs)) if got[i] != base[i]]
    print(env, "differing docs:", bad)
    if bad:
        a = json.dumps(base[bad[0]], indent=1).splitlines()
        b = json.dumps(got[bad[0]], indent=1).splitlines()
        print("\n".join(list(difflib.unified_diff(a, b, lineterm="", n=2))[:60]))
