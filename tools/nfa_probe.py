"""Launches the NFA regex pack (tests/golden/nfa_rulepack: regexes past the DFA limits, evaluated by the NFA
kernel variant) over a synthetic corpus, for counter passes (rocprofv3 --pmc ... -- python3 tools/nfa_probe.py):
the LDS bank conflicts of the staged NFA tables.  Prints the kernel ms of each launch."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd")]
import guard_amd  # noqa: E402


def docs(n, seed=5150):
    r = random.Random(seed)
    cjk = "".join(chr(0x4E00 + 3 * k) for k in range(260))
    out = []
    for _ in range(n):
        res = {}
        for k in range(3):
            m = r.choice([5, 12, 13, 14, 16, 25])
            props = {"Code": r.choice(["", "c", "q"]) + "".join(r.choice("ab") for _ in range(m))}
            if r.random() < 0.7:
                lab = "".join(r.choice(cjk) for _ in range(r.choice([1, 2, 3, 6])))
                props["Label"] = r.choice([lab, "x" + lab + "y", lab + "!", "ab" + lab])
            res["r%d" % k] = {"Type": "AWS::S3::Bucket", "Properties": props}
        out.append(json.dumps({"Resources": res}, ensure_ascii=False))
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    p = os.path.join(ROOT, "tests", "golden", "nfa_rulepack")
    s = guard_amd.Session()
    for f in sorted(os.listdir(p)):
        if f.endswith(".guard"):
            s.add_rules(open(os.path.join(p, f)).read(), f)
    d = docs(n)
    s.add_docs(d, ["n%d.json" % i for i in range(n)], threads=16)
    s.upload()
    s.set_option("rx_memo_per_launch", True)
    print(json.dumps({"docs": n, "kernel_ms": s.eval(3)}))
    s.close()


if __name__ == "__main__":
    main()
