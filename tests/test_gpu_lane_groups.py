"""Lane groups: G lanes per document run its tile in step and split every chunk
of its filtered list fan-outs -- the reference's per-element Filter (eval_context.rs:723-828) and
check_and_delegate over map values (:268-313) -- merging the verdicts with shuffles (eval_recursive.inc
coop_chunk).  Whatever G, the bytes equal the oracle's and the one-lane-per-tile kernel's; an error raised
inside a cooperatively tested filter surfaces as the reference raises it."""
import json
import os

import pytest

import guard_amd
import synth
from guard_oracle import validate_structured as oracle_validate
from rulepack import rule_pack

pytestmark = pytest.mark.gpu


def _report(rules, docs, group, prefix="g", output="json"):
    old = os.environ.get("GG_LANE_GROUP")
    if group is None:
        os.environ.pop("GG_LANE_GROUP", None)
    else:
        os.environ["GG_LANE_GROUP"] = str(group)
    try:
        s = guard_amd.Session()
        try:
            for name, text in rules:
                s.add_rules(text, name)
            s.add_docs(docs, ["%s-%d.json" % (prefix, i) for i in range(len(docs))])
            s.eval(1)
            g = s.stat(s.STAT["lane_group"])
            return s.report(output), g
        finally:
            s.close()
    finally:
        if old is None:
            os.environ.pop("GG_LANE_GROUP", None)
        else:
            os.environ["GG_LANE_GROUP"] = old


@pytest.mark.parametrize("group", [2, 16, 64])
def test_terraform_plans_every_group_size_vs_oracle(group):
    rules = rule_pack("cfg4")
    docs = synth.tf_corpus(9, start=300, n_resources=150) + synth.tf_corpus(2, start=900, n_resources=700)
    data = [("g-%d.json" % i, d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    (out, code), g = _report(rules, docs, group)
    assert g == group
    assert (out, code) == (exp, ecode)


def test_full_size_plans_pick_lane_groups():
    """a launch of few large plans selects lane groups by itself (capi.cpp session_upload)"""
    rules = rule_pack("cfg4")
    docs = synth.tf_corpus(3, start=40, n_resources=2000)
    data = [("g-%d.json" % i, d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    (out, code), g = _report(rules, docs, None)
    assert g > 1
    assert (out, code) == (exp, ecode)
    assert _report(rules, docs, 1)[0] == (exp, ecode)


@pytest.mark.parametrize("group", [4, 32])
def test_cfn_templates_in_lane_groups(group):
    """groups on CloudFormation templates (map fan-outs, type blocks, fast filters) and the cfg3 pack"""
    for pack, docs in (("cfg2", synth.cfn_corpus(40, start=11, n_resources=20)),
                       ("cfg3", synth.cfn_corpus(20, start=77, n_resources=30))):
        rules = rule_pack(pack)
        base, _ = _report(rules, docs, 1)
        (out, code), g = _report(rules, docs, group)
        assert g == group
        assert (out, code) == base, pack


def test_formats_in_lane_groups():
    rules = rule_pack("cfg4")
    docs = synth.tf_corpus(4, start=5, n_resources=90)
    for fmt in ("yaml", "sarif", "junit"):
        assert _report(rules, docs, 8, output=fmt)[0] == _report(rules, docs, 1, output=fmt)[0], fmt


def test_size_order_does_not_change_the_report():
    """lane-group launches evaluate documents largest first inside each XCD's share (capi.cpp session_upload,
    GG_SIZE_ORDER); the report stays in document order and equals load order's and the oracle's"""
    rules = rule_pack("cfg4")
    sizes = [40, 260, 90, 700, 15, 330, 120, 520, 60, 210, 410, 25, 150, 95, 380, 45, 600, 70]
    docs = [synth.tf_corpus(1, start=31 + i, n_resources=n)[0] for i, n in enumerate(sizes)]
    data = [("g-%d.json" % i, d) for i, d in enumerate(docs)]
    exp = oracle_validate(rules, data)[:2]
    old = os.environ.get("GG_SIZE_ORDER")
    try:
        os.environ["GG_SIZE_ORDER"] = "0"
        unsorted = _report(rules, docs, 16)[0]
    finally:
        if old is None:
            os.environ.pop("GG_SIZE_ORDER", None)
        else:
            os.environ["GG_SIZE_ORDER"] = old
    assert _report(rules, docs, 16)[0] == exp
    assert unsorted == exp


RAISING = """let picked = items[ size empty ]
rule r when %picked !empty {
    %picked.name exists
}
"""


def test_error_inside_a_cooperative_filter():
    """`empty` on an integer raises inside the filter (eval.rs:251-262): the chunk goes back to the
    sequential tests, which raise the reference's error for the first such element in order"""
    items = [{"name": "a%d" % k, "size": ([] if k % 5 else "s")} for k in range(150)]
    items[97]["size"] = 7   # the first element whose test raises
    items[140]["size"] = 9
    doc = json.dumps({"items": items})
    rules = [("raise.guard", RAISING)]
    data = [("g-0.json", doc)]
    try:
        oracle_validate(rules, data, raise_errors=True)
        raise AssertionError("the oracle did not abort")
    except Exception as e:   # guard_oracle.GuardError
        want = getattr(e, "display", lambda: str(e))()
    for group in (1, 16, 64):
        with pytest.raises(guard_amd.GuardError) as g:
            _report(rules, [doc], group)
        assert g.value.message == want, group


BLOCKS = """rule values_block {
    items[*] {
        v == 1
        w exists
        tags[*] != 'bad'
    }
}
rule filtered_block_or {
    items[ kind == 'a' ] {
        v == 1 or w == 2
    }
}
rule missing_values_block {
    Resources.*.Properties {
        Name exists
    }
}
rule nested_block {
    items[*] {
        tags[*] { this != 'bad' }
    }
}
"""


def _block_doc(n, seed):
    r = seed
    items, res = [], {}
    for k in range(n):
        r = (r * 1103515245 + 12345) & 0x7FFFFFFF
        it = {"kind": "ab"[r % 2], "v": (r >> 3) % 2, "tags": ["ok", "bad"][: 1 + (r >> 5) % 2]}
        if (r >> 7) % 3:
            it["w"] = (r >> 9) % 3
        items.append(it)
        res["r%d" % k] = {"Type": "T"} if (r >> 11) % 4 == 0 else {"Type": "T", "Properties": {"Name": "x"} if (r >> 13) % 2 else {}}
    return json.dumps({"items": items, "Resources": res})


@pytest.mark.parametrize("n", [5, 150, 700, 3000])
def test_split_blocks_vs_oracle(n):
    """block clauses over a document's values evaluated by the lane group at once (eval_recursive.inc split_block):
    the reference's records in value order -- failing clauses, missing block values, disjunctions, nested blocks --
    and, past the record staging (n = 3000), the wave kernel's retry, for every group size"""
    rules = [("blocks.guard", BLOCKS)]
    docs = [_block_doc(n, 17 + n), _block_doc(n // 2 + 1, 5 + n)]
    data = [("g-%d.json" % i, d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    for group in (1, 16, 64):
        (out, code), g = _report(rules, docs, group)
        assert g == group
        assert (out, code) == (exp, ecode), group


RAISING_BLOCK = """rule r {
    items[*] {
        name exists
        size empty
    }
}
"""


def test_error_inside_a_split_block():
    """an error raised by one value of a split block: the sequential loop runs again and raises the reference's
    error for the first such value"""
    items = [{"name": "a%d" % k, "size": []} for k in range(150)]
    items[61]["size"] = 7
    items[120]["size"] = 9
    doc = json.dumps({"items": items})
    rules = [("raise.guard", RAISING_BLOCK)]
    try:
        oracle_validate(rules, [("g-0.json", doc)], raise_errors=True)
        raise AssertionError("the oracle did not abort")
    except Exception as e:   # guard_oracle.GuardError
        want = getattr(e, "display", lambda: str(e))()
    for group in (1, 16, 64):
        with pytest.raises(guard_amd.GuardError) as g:
            _report(rules, [doc], group)
        assert g.value.message == want, group


COMPARES = """rule eq_values { items[*].v == 1 }
rule ne_lists { items[*].tags != 'bad' }
rule exists_values { items[*].w exists }
rule in_values { items[*].kind in ['a', 'c'] }
rule in_lists { items[*].tags in ['ok'] }
rule gt_values { items[*].v > 0 }
rule regex_values { items[*].name == /^n[0-4]/ }
rule some_values { some items[*].w == 2 }
rule not_in_values { items[*].kind not in ['b'] }
rule empty_values { items[*].tags !empty }
"""


@pytest.mark.parametrize("n", [40, 700, 3000])
def test_split_comparisons_vs_oracle(n):
    """an access clause's comparison over a long value list shared out by the lane group (eval_recursive.inc
    split_compare): unresolved values' records first, then each value's comparison, in value order -- equal to
    the oracle for every group size, past the record staging too (n = 3000)"""
    rules = [("compares.guard", COMPARES)]
    docs = [_block_doc(n, 31 + n), _block_doc(n // 3 + 1, 3 + n)]
    data = [("g-%d.json" % i, d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    for group in (1, 16, 64):
        (out, code), g = _report(rules, docs, group)
        assert g == group
        assert (out, code) == (exp, ecode), group
