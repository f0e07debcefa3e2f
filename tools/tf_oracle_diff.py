"""Diagnostic: the cfg4 pack's lane-kernel report (G = 1, 2, 16) against the oracle, first differing document."""
import difflib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import guard_amd  # noqa: E402
import rulepack  # noqa: E402
import synth  # noqa: E402
from guard_oracle import validate_structured as oracle_validate  # noqa: E402

rules = rulepack.rule_pack("cfg4")
docs = synth.tf_corpus(9, start=300, n_resources=150) + synth.tf_corpus(2, start=900, n_resources=700)
exp = json.loads(oracle_validate(rules, [("g-%d.json" % i, d) for i, d in enumerate(docs)])[0])
for g in ("1", "2", "16"):
    os.environ["GG_LANE_GROUP"] = g
    s = guard_amd.Session()
    for n, t in rules:
        s.add_rules(t, n)
    s.add_docs(docs, ["g-%d.json" % i for i in range(len(docs))])
    s.eval(1)
    got = json.loads(s.report()[0])
    print("errors", s.stat(s.STAT["errors"]), "first_error", s.stat(s.STAT["first_error"]), "retried", s.stat(s.STAT["retried"]))
    s.close()
    bad = [i for i in range(len(docs)) if got[i] != exp[i]]
    print("G", g, "differing docs:", bad)
    for i in bad[:2]:
        print(" doc", i, "oracle", [(r["Rule"]["name"], len(r["Rule"]["checks"])) for r in exp[i]["not_compliant"]])
        print(" doc", i, "gpu   ", [(r["Rule"]["name"], len(r["Rule"]["checks"])) for r in got[i]["not_compliant"]])
    if bad:
        a = json.dumps(exp[bad[0]], indent=1).splitlines()
        b = json.dumps(got[bad[0]], indent=1).splitlines()
        print("\n".join(list(difflib.unified_diff(a, b, "oracle", "gpu", lineterm="", n=3))[:80]))
