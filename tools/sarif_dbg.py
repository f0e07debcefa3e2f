import os, sys
sys.path[:0] = ["tests", "oracle", "cloudformation-guard_amd"]
os.environ["GG_RESIDENT_ARENA"] = "1"
import guard_amd, synth
from rulepack import rule_pack
from guard_oracle import validate_structured as oracle_validate
rules = rule_pack("cfg2")
docs = synth.cfn_corpus(300, start=4321, n_resources=25)
data = [("r-%d.json" % i, d) for i, d in enumerate(docs)]
for order in (["sarif"], ["yaml", "sarif"]):
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    st = s.add_docs_device(docs, ["r-%d.json" % i for i in range(len(docs))])
    s.eval(1)
    s.set_device_report(True)
    for fmt in order:
        out, code = s.report(fmt)
        e, c, _ = oracle_validate(rules, data, output=fmt)
        if out != e:
            i = next(k for k in range(min(len(out), len(e))) if out[k] != e[k]) if out[:min(len(out),len(e))] != e[:min(len(out),len(e))] else min(len(out), len(e))
            print(order, fmt, "DIFF at", i, "len", len(out), len(e))
            print("GOT:", repr(out[max(0,i-300):i+200]))
            print("EXP:", repr(e[max(0,i-300):i+200]))
        else:
            print(order, fmt, "OK")
    s.close()
