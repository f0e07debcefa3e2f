"""Rule packs of the BASELINE.json workloads:
  cfg2 -- reference rule files from guard-examples/encryption and guard/resources/validate/rules-dir
          plus two pack-local files (tests/golden/rulepack, 7 files);
  cfg3 -- the full-registry stand-in: every in-scope .guard file of the reference
          (tests/golden/cfg3_rulepack, 22 files);
  cfg4 -- Terraform plan rules (tests/golden/tf_rulepack);
  cfg5 -- network-reachability regex / join rules (tests/golden/net_rulepack)."""
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PACKS = {"cfg2": "rulepack", "cfg3": "cfg3_rulepack", "cfg4": "tf_rulepack", "cfg5": "net_rulepack"}
G = os.path.join(GOLDEN, "rulepack")


def rule_pack(name="cfg2"):
    d = os.path.join(GOLDEN, PACKS[name])
    return [(f, open(os.path.join(d, f)).read()) for f in sorted(os.listdir(d)) if f.endswith(".guard")]
