"""Per-rules-file kernel cost on the cfg-2 corpus (diagnostic; not the headline bench)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import rulepack  # noqa: E402

ndocs = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
out = {}
for name, text in rulepack.rule_pack():
    s = guard_amd.Session()
    s.add_rules(text, name)
    s.add_synthetic(0, ndocs, threads=16)
    s.upload()
    ms = s.eval(3)
    out[name] = {"kernel_ms": round(min(ms), 3), "us_per_tile": round(min(ms) * 1e3 / ndocs, 3),
                 "records": s.stat(8), "fail_pass_skip_err": [s.stat(4), s.stat(5), s.stat(6), s.stat(7)],
                 "first_error": s.stat(10)}
    s.close()
print(json.dumps(out, indent=1))
