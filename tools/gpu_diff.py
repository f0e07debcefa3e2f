"""Debug helper: run the reference test specs on the GPU and dump mismatches vs the oracle."""
import difflib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
from guard_oracle import validate_structured as oracle_validate  # noqa: E402

cases = json.load(open(os.path.join(ROOT, "tests", "golden", "expectations.json")))
out_lines = []
nbad = 0
for c in cases:
    rules = [(c["rules_name"], c["rules_text"])]
    data = [("input-%d.json" % c["case"], c["input_json"])]
    exp, ecode, eerr = oracle_validate(rules, data)
    try:
        got, code = guard_amd.validate_structured(rules, data)
    except guard_amd.GuardError as e:
        got, code = "ERR %d %s" % (e.code, e.message), -1
    if got != exp or code != ecode:
        nbad += 1
        out_lines.append("=== %s case %d: code %d vs %d" % (c["spec"], c["case"], code, ecode))
        if got.startswith("ERR"):
            out_lines.append(got)
        else:
            d = list(difflib.unified_diff(exp.splitlines(), got.splitlines(), lineterm="", n=2))
            out_lines.extend(d[:40])
out_lines.append("bad %d of %d" % (nbad, len(cases)))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
open(os.path.join(ROOT, "gpurun_out", "gpu_diff.txt"), "w").write("\n".join(out_lines))
print("\n".join(out_lines[-5:]))
