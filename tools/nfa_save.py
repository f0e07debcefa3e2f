"""Diagnostic: the NFA pack's raw results (tiles, rule statuses, records) from the lane and wave kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import guard_amd  # noqa: E402
import test_gpu_parity as t  # noqa: E402

p = os.path.join(ROOT, "tests", "golden", "nfa_rulepack")
rules = [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
data = [("n%d.json" % i, d) for i, d in enumerate(t._nfa_docs())]
out = sys.argv[1]
for mode in (0, 1):
    s = guard_amd.Session()
    s.configure(mode, 0)
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs([x for _, x in data], [n for n, _ in data])
    s.eval(1)
    s.save_results(os.path.join(out, "nfa_mode%d.bin" % mode))
    print("mode", mode, "errors", s.stat(s.STAT["errors"]), "retried", s.stat(s.STAT["retried"]), "records", s.stat(s.STAT["records"]))
    s.close()
