"""Micro-benchmarks of single rule shapes on the cfg-2 corpus (diagnostic)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from micro_cases import CASES  # noqa: E402
ndocs = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
s = guard_amd.Session()
for k, v in CASES.items():
    s.add_rules(v, k + ".guard")
s.add_synthetic(0, ndocs, threads=16)
s.upload()
s.eval(1)
out = {}
for i, k in enumerate(CASES):
    t = guard_amd.Session()
    t.add_rules(CASES[k], k + ".guard")
    t.add_synthetic(0, ndocs, threads=16)
    t.upload()
    ms = t.eval(3)
    out[k] = {"kernel_ms": round(min(ms), 3), "records": t.stat(8), "fail_pass_skip_err": [t.stat(4), t.stat(5), t.stat(6), t.stat(7)]}
    t.close()
print(json.dumps(out, indent=1))
