"""The oracle's console (non-structured) `cfn-guard validate` reporters against the reference's
goldens (guard/tests/validate.rs:237-345, 405-418, 488-540; resources/validate/output-dir/*.out)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import console_cases  # noqa: E402
from guard_oracle.console import ReadCursor, summary_flags, validate_console  # noqa: E402

CASES = console_cases.cases()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_console_golden(case):
    name, rules, data, opts, expected, code, _ = case
    out, rc, err = validate_console(rules, data, **opts)
    assert rc == code, err
    if expected is not None:
        assert out == expected


def test_payload_type_block_over_nothing_is_an_evaluation_error():
    # validate.rs:555-564: exit INTERNAL_FAILURE, nothing on stdout
    rules, data = console_cases._payload(console_cases.PAYLOAD_TYPE_BLOCK)
    out, rc, err = validate_console(rules, data)
    assert (out, rc) == ("", -1)
    assert "Unable to resolve type block query: d1z::Y" in err


def test_summary_flags_fold():
    # validate.rs:254-268: `none` resets the fold, later values still add
    assert summary_flags(["fail"]) == 2
    assert summary_flags(["none", "fail"]) == 2
    assert summary_flags(["fail", "none"]) == 0
    assert summary_flags(["all"]) == 7


def test_read_cursor_backward_seek_numbering():
    # utils/mod.rs:46-64: a forward seek from a position reached by seeking back records the lines
    # it reads under the cursor's running number
    c = ReadCursor("".join("l%d\n" % i for i in range(1, 31)))
    assert c.seek_line(11) == (11, "l11")
    for _ in range(5):
        c.next()
    assert c.seek_line(3) == (3, "l3")
    for _ in range(5):
        c.next()                        # line_num 8, 16 lines read
    assert c.seek_line(16) == (16, "l16")
    assert c.next() == (9, "l17")       # the entry the forward seek pushed as line 9
    # a seek target at exactly the lines read runs to the end
    d = ReadCursor("a\nb\nc\n")
    d.seek_line(2); d.next()
    assert d.seek_line(3) is None


def test_parse_error_and_exit_code_order():
    # evaluate_rule: a rules file that does not parse -> stderr + 5; the last non-zero code wins
    rules = [("bad.guard", "rule {"), ("ok.guard", "rule r { Resources exists }")]
    data = [("d.json", '{"Resources": {}}')]
    out, rc, err = validate_console(rules, data)
    assert rc == 0 or rc == 5
    assert err.startswith("Parsing error handling rule file = bad.guard, Error = ")
    assert rc == 5
