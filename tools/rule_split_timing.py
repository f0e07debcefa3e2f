"""Kernel time of each rule of a pack on its own (diagnostic): the pack's `let` lines plus one rule per
session, over the cfg-4 bench corpus (or PACK=cfg2/cfg5), min of 3 evaluations.  Shows which rule
shapes the lane kernel spends its time on.  Usage: PACK=cfg4 python tools/rule_split_timing.py [docs]"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import rulepack  # noqa: E402
import synth  # noqa: E402


def split_rules(text):
    """(preamble: everything before the first rule -- the lets, multi-line ones too; [rule blocks])"""
    lines = text.splitlines()
    first = next(i for i, l in enumerate(lines) if l.startswith("rule "))
    rules, cur = [], None
    for line in lines[first:]:
        if cur is None:
            if line.startswith("rule "):
                cur = [line]
        else:
            cur.append(line)
            if line.startswith("}"):
                rules.append("\n".join(cur))
                cur = None
    return lines[:first], rules


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    pack = os.environ.get("PACK", "cfg4")
    if os.environ.get("SIZE"):   # n plans of one size (SIZE=2000, n=1: the latency of the largest bench plan)
        corpus = synth.tf_corpus(n, n_resources=int(os.environ["SIZE"]))
    else:
        corpus = synth.tf_bench_corpus(n) if pack == "cfg4" else synth.config_corpus(n)
    names = ["d-%d.json" % i for i in range(n)]
    out = {}
    groups = [int(g) for g in os.environ.get("GSIZES", "16").split(",")]
    files = rulepack.rule_pack(pack)
    if os.environ.get("EXTRA"):   # a guard file of variant rules (lets first), each rule timed on its own
        files = [(os.path.basename(os.environ["EXTRA"]), open(os.environ["EXTRA"]).read())]
    for fname, text in files:
        lets, rules = split_rules(text)
        variants = [("(whole file)", text)] + [(re.match(r"rule (\w+)", r).group(1), "\n".join(lets) + "\n" + r + "\n")
                                              for r in rules]
        for (name, body), g in [(v, g) for v in variants for g in groups]:
            os.environ["GG_LANE_GROUP"] = str(g)
            name = "%s@G%d" % (name, g)
            s = guard_amd.Session()
            try:
                s.add_rules(body, fname)
                s.add_docs(corpus, names, threads=16)
                s.upload()
                ms = min(s.eval(3))
                out["%s:%s" % (fname, name)] = {"ms": round(ms, 2), "group": s.stat(s.STAT["lane_group"])}
            finally:
                s.close()
            print(json.dumps({"rule": "%s:%s" % (fname, name), **out["%s:%s" % (fname, name)]}), flush=True)


if __name__ == "__main__":
    main()
