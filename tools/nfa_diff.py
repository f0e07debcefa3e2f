"""Diagnostic: the NFA regex pack's report vs the oracle's, first differing lines (lane and wave kernels)."""
import difflib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import guard_amd  # noqa: E402
from guard_oracle import validate_structured as oracle_validate  # noqa: E402
import test_gpu_parity as t  # noqa: E402

p = os.path.join(ROOT, "tests", "golden", "nfa_rulepack")
rules = [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
data = [("n%d.json" % i, d) for i, d in enumerate(t._nfa_docs())]
exp, ecode, _ = oracle_validate(rules, data)
for mode in (0, 1):
    s = guard_amd.Session()
    s.configure(mode, 0)
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs([x for _, x in data], [n for n, _ in data])
    s.eval(1)
    out, code = s.report("json")
    s.close()
    print("mode", mode, "equal", out == exp, code, ecode)
    if os.environ.get("DUMP"):
        open(os.path.join(os.environ["DUMP"], "gpu_mode%d.json" % mode), "w").write(out)
        open(os.path.join(os.environ["DUMP"], "oracle.json"), "w").write(exp)
    if out != exp:
        d = list(difflib.unified_diff(exp.splitlines(), out.splitlines(), "oracle", "gpu", n=8, lineterm=""))
        print("\n".join(d[:120]))
