"""Builds tests/golden/verbose_golden.json: the reference's one golden for guard-ffi
`run_checks(..., verbose = true)` -- the serde EventRecord tree pinned by
guard/tests/functional.rs:7-160 (test_run_check): its data document, its rule text, the data / rules
file names it passes and the expected tree (compared as parsed JSON values, as that test does).
Run once in the build container:
    python tests/golden/make_verbose_cases.py /root/reference
"""
import json
import os
import re
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = os.path.join(ROOT, "guard", "tests", "functional.rs")


def main():
    text = open(SRC, encoding="utf-8").read()
    raws = re.findall(r'r#"(.*?)"#', text, re.S)          # the data document, then the expected tree
    rule = re.search(r'let rule = "((?:[^"\\]|\\.)*)";', text).group(1)
    rule = json.loads('"' + rule + '"')                    # Rust escapes used here (\") are JSON's
    names = re.findall(r'file_name: "([^"]+)"', text)
    data, expected = raws[0], raws[1]
    case = {"src": "guard/tests/functional.rs:7-160", "data": data, "data_name": names[0],
            "rules": rule, "rules_name": names[1], "expected": json.loads(expected)}
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "verbose_golden.json")
    with open(out, "w", encoding="utf-8") as f:
        json.dump([case], f, indent=1, ensure_ascii=False)
        f.write("\n")
    print("wrote", out)


if __name__ == "__main__":
    main()
