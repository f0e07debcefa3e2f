"""Child process of tests/test_gpu_machine.py: with GG_LIB pointing at the machine build
(libcfnguard_mi355x_machine.so, csrc/eval_machine.inc), evaluates rule packs over corpora and compares every
report with the CPU oracle.  Prints one line per case; exits 1 on the first mismatch."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "oracle"), os.path.join(os.path.dirname(HERE), "cloudformation-guard_amd")]
import guard_amd  # noqa: E402
import synth  # noqa: E402
from guard_oracle import validate_structured as oracle_validate  # noqa: E402
from rulepack import rule_pack  # noqa: E402

G = os.path.join(HERE, "golden")


def pack(name):
    p = os.path.join(G, name)
    return [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]


def main():
    assert guard_amd.LIB_PATH.endswith("_machine.so"), guard_amd.LIB_PATH
    cases = [
        ("cfg2", rule_pack("cfg2"), [("s%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(200, start=9, n_resources=25))]),
        ("cfg3", rule_pack("cfg3"), [("t%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(60, start=90, n_resources=20))]),
        ("cfg4", pack("tf_rulepack"), [("p%d.json" % i, d) for i, d in enumerate(synth.tf_corpus(6, start=3, n_resources=40))]),
        ("cfg5", rule_pack("cfg5"), [("c%d.json" % i, d) for i, d in enumerate(synth.config_corpus(60, start=5))]),
    ]
    for name in ("capture_rulepack", "edge_rulepack", "ops_rulepack", "count_rulepack", "conv_rulepack", "nfa_rulepack",
                 "wordb_rulepack"):
        if os.path.isdir(os.path.join(G, name)) and any(f.endswith(".guard") for f in os.listdir(os.path.join(G, name))):
            cases.append((name, pack(name), [("d%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(40, start=700, n_resources=12))]))
    for name, rules, data in cases:
        for fmt in ("json", "sarif"):
            exp, ecode, _ = oracle_validate(rules, data, output=fmt)
            got = guard_amd.validate_structured(rules, data, output=fmt)
            if got != (exp, ecode):
                print("MISMATCH", name, fmt, flush=True)
                sys.exit(1)
        print("ok", name, flush=True)


if __name__ == "__main__":
    main()
