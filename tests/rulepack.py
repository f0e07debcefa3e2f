"""The cfg-2 rule pack (BASELINE.json configs[1]): reference rule files from
guard-examples/encryption and guard/resources/validate/rules-dir plus two pack-local files."""
import os

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rulepack")


def rule_pack():
    return [(f, open(os.path.join(G, f)).read()) for f in sorted(os.listdir(G)) if f.endswith(".guard")]
