"""Collects the regex literals of every .guard file in the reference (guard-examples/, guard/resources/)
into tests/golden/regex_patterns.json (data fixture; run once in the build container):
    python tests/golden/make_regex_cases.py /root/reference
"""
import json
import os
import re
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
# a regex literal in the Guard DSL: /.../ after an operator or list bracket (parser.rs parse_regex)
RX = re.compile(r"(?:==|!=|IN|in|\[|,|<<)\s*/((?:[^/\\\n]|\\.)+)/")


def main():
    pats = set()
    for d, _, files in os.walk(ROOT):
        for f in files:
            if f.endswith(".guard"):
                for m in RX.finditer(open(os.path.join(d, f), encoding="utf-8", errors="replace").read()):
                    pats.add(m.group(1).replace("\\/", "/"))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "regex_patterns.json")
    json.dump(sorted(pats), open(out, "w"), indent=1)
    print(len(pats), "patterns ->", out)


if __name__ == "__main__":
    main()
