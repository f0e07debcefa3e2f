"""Quick filters (eval_core.inc quick_conj; compiler.cpp quick_conj): list filters whose clauses are key paths
(an unnamed `[*]` last) against one literal, or unary checks, tested per value without the evaluator's calls --
the reference's Filter over a list (eval_context.rs:723-828) with each clause evaluated as eval_access does
(eval.rs:1040-1225).  The bytes equal the oracle's with one lane per document and in lane groups, including the
values binary_literal_stream leaves to the generic test (IN over a list value) and case-converted keys."""
import json

import pytest

import guard_amd
from guard_oracle import validate_structured as oracle_validate

pytestmark = pytest.mark.gpu

RULES = """rule kind_eq { items[ kind == 'a' ].name == /^n/ }
rule int_eq { items[ v == 1 ].name exists }
rule list_any { items[ tags[*] == 'ok' ].v == 1 }
rule list_ne { items[ tags[*] != 'bad' ].v >= 0 }
rule path_in { items[ a.b.c in ['x', 'y'] ].kind == 'a' }
rule exists_f { items[ w exists ].w < 2 }
rule not_exists_f { items[ w !exists ].kind == 'b' }
rule is_list_f { items[ tags is_list ].name exists }
rule or_f { items[ kind == 'a' or v == 1 ].w exists }
rule some_f { items[ some tags[*] == 'bad' ].v == 0 }
rule gt_f { items[ v > 0 ].kind in ['a', 'b'] }
rule regex_f { items[ name == /^n1/ ].v == 1 }
rule list_in_f { items[ tags in ['ok'] ].name exists }
rule two_clauses { items[ kind == 'b'
                          v == 0 ].tags[*] == 'ok' }
rule nested_list { items[ grid[*] == 'x' ].name exists }
rule converted_key { items[ kindName == 'z' ].name exists }
rule empty_result { items[ kind == 'nope' ].name exists }
"""


def _doc(n, seed):
    r = seed
    items = []
    for k in range(n):
        r = (r * 1103515245 + 12345) & 0x7FFFFFFF
        it = {"name": "n%d" % k, "kind": "abc"[r % 3], "v": (r >> 3) % 3,
              "tags": [["ok"], ["ok", "bad"], [], "ok"][(r >> 5) % 4]}
        if (r >> 7) % 3:
            it["w"] = (r >> 9) % 3
        if (r >> 11) % 2:
            it["a"] = {"b": {"c": "xyz"[(r >> 12) % 3]}}
        elif (r >> 13) % 2:
            it["a"] = {"b": 5}
        it["grid"] = [["x"], "x", "y", {"x": 1}, []][(r >> 14) % 5]
        if (r >> 17) % 4 == 0:
            it["kind_name" if (r >> 19) % 2 else "KindName"] = "z"
        items.append(it)
    return json.dumps({"items": items})


def _report(rules, docs, group):
    import os
    old = os.environ.get("GG_LANE_GROUP")
    os.environ["GG_LANE_GROUP"] = str(group)
    try:
        s = guard_amd.Session()
        try:
            for name, text in rules:
                s.add_rules(text, name)
            s.add_docs(docs, ["q-%d.json" % i for i in range(len(docs))])
            s.eval(1)
            return s.report()
        finally:
            s.close()
    finally:
        if old is None:
            os.environ.pop("GG_LANE_GROUP", None)
        else:
            os.environ["GG_LANE_GROUP"] = old


@pytest.mark.parametrize("group", [1, 16])
def test_quick_filters_vs_oracle(group):
    rules = [("quick.guard", RULES)]
    docs = [_doc(n, 7 + n) for n in (1, 40, 150, 300)]
    exp, ecode, _ = oracle_validate(rules, [("q-%d.json" % i, d) for i, d in enumerate(docs)])
    assert _report(rules, docs, group) == (exp, ecode)
