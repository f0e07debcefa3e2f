"""Generate tests/golden/expectations.json from the reference's own `cfn-guard test` specs.

Run in the build container only (needs /root/reference).  Each reference spec file
(guard-examples/**/*-tests.yaml and guard/resources/test-command/**) pairs a rules file with
inputs and expected per-rule statuses.  The spec `input` is loaded the way the reference's
test command loads it (serde_yaml -> PathAwareValue, commands/test.rs:480-484) and re-emitted
as compact JSON so both the oracle and the MI355X path consume it as a data document.
Output: data only (rules text, input JSON, expected statuses).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from guard_oracle.loader import load_serde_yaml_tree, serde_tree_to_pv, pv_to_json_text  # noqa: E402
from guard_oracle.pv import LIST, MAP  # noqa: E402

REF = "/root/reference"
PAIRS = []
for root, _, files in os.walk(os.path.join(REF, "guard-examples")):
    for f in files:
        if f.endswith("-tests.yaml"):
            rules = os.path.join(root, f.replace("-tests.yaml", ".guard"))
            if os.path.exists(rules):
                PAIRS.append((rules, os.path.join(root, f)))
TC = os.path.join(REF, "guard/resources/test-command")
PAIRS += [
    (os.path.join(TC, "dir/s3_bucket_logging_enabled.guard"), os.path.join(TC, "dir/tests/s3_bucket_logging_enabled_tests.yaml")),
    (os.path.join(TC, "dir/s3_bucket_server_side_encryption_enabled.guard"), os.path.join(TC, "dir/tests/s3_bucket_server_side_encryption_enabled.json")),
    (os.path.join(TC, "dir/s3_bucket_logging_enabled.guard"), os.path.join(TC, "data-dir/s3_bucket_logging_enabled_tests.yaml")),
    (os.path.join(TC, "dir/s3_bucket_server_side_encryption_enabled.guard"), os.path.join(TC, "data-dir/s3_bucket_server_side_encryption_enabled.yaml")),
]

cases = []
for rules_path, spec_path in sorted(PAIRS):
    spec = serde_tree_to_pv(load_serde_yaml_tree(open(spec_path).read()))
    assert spec.kind == LIST
    for i, case in enumerate(spec.val):
        inp = case.val.values.get("input")
        exp = case.val.values["expectations"].val.values["rules"]
        cases.append({
            "rules_name": os.path.basename(rules_path),
            "rules_text": open(rules_path).read(),
            "spec": os.path.relpath(spec_path, REF),
            "case": i,
            "input_json": pv_to_json_text(inp) if inp is not None else "{}",
            "expected": {k: v.val for k, v in exp.val.values.items()},
        })
json.dump(cases, open(os.path.join(HERE, "expectations.json"), "w"), indent=1, ensure_ascii=False)
print(len(cases), "cases")
