"""Diagnostic: which NFA rules differ from the oracle in the lane kernel, rule by rule."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import guard_amd  # noqa: E402
from guard_oracle import validate_structured as oracle_validate  # noqa: E402
import test_gpu_parity as t  # noqa: E402
import rule_split_timing as rs  # noqa: E402

p = os.path.join(ROOT, "tests", "golden", "nfa_rulepack", "nfa.guard")
pre, rules = rs.split_rules(open(p).read())
data = [("n%d.json" % i, d) for i, d in enumerate(t._nfa_docs())]
J = "\n".join
variants = [("r0-2", J(rules[:3])), ("r0-3", J(rules[:4])), ("all", J(rules)), ("r1-4", J(rules[1:])), ("r2-4", J(rules[2:])),
            ("r0,r1,r3", J([rules[0], rules[1], rules[3]])), ("r2,r3", J(rules[2:4]))]
for name, body in variants:
    rr = [("nfa.guard", body + "\n")]
    exp, ecode, _ = oracle_validate(rr, data)
    s = guard_amd.Session()
    s.configure(0, 0)
    s.add_rules(body + "\n", "nfa.guard")
    s.add_docs([x for _, x in data], [n for n, _ in data])
    s.eval(1)
    out, code = s.report("json")
    print(name, out == exp, s.stat(s.STAT["retried"]))
    s.close()
