"""The error half of the drop-in contract on the MI355X path: evaluation errors that abort a run
must carry the reference's guard-ffi code (guard-ffi/src/errors.rs:12-38) and Error Display text
(guard/src/rules/errors.rs:11-54), exactly as the oracle raises them; exit-code precedence of
rules-file parse errors (structured.rs:40-43, 110-112; reporters/mod.rs:97-103; xml.rs:62-66)."""
import json

import pytest

import guard_amd
from guard_oracle import validate_structured as oracle_validate
from guard_oracle import run_checks as oracle_run_checks
from guard_oracle.errors import GuardError, FFI_CODES

pytestmark = pytest.mark.gpu

DOC = json.dumps({"Resources": {"b": {"Type": "AWS::S3::Bucket",
                                      "Properties": {"Port": 8080, "Name": "x", "F": 1.5, "N": None}}},
                  "Keys": {"k": 5, "l": ["b", 3], "s": "b"}})

# (name, rules text, data text): every one aborts the reference's evaluation
ABORTS = [
    ("empty-int", "Resources.*.Properties.Port empty", DOC),                  # eval.rs:251-262
    ("empty-float", "Resources.*.Properties.F !empty", DOC),
    ("empty-null", "Resources.*.Properties.N empty", DOC),
    ("var-missing", "%nothere exists", DOC),                                  # eval_context.rs:1131
    ("rule-missing", "rule r {\n  missing_rule\n}", DOC),                     # eval_context.rs:1098-1104
    ("param-arity", "rule p(a, b) { %a exists }\nrule r { p(Resources) }", DOC),   # eval.rs:1588-1596
    ("param-missing", "rule r { nope(Resources) }", DOC),                     # eval_context.rs:1082-1086
    ("interp-non-string", "let k = Keys.k\nrule r { Resources.%k exists }", DOC),   # eval_context.rs:508-518
    ("interp-list-non-string", "let k = Keys.l\nrule r { Resources.%k exists }", DOC),
    ("interp-query", "let k = 'b'\nrule r { Resources.%k.* exists }", DOC),  # eval_context.rs:441-443
    ("typeblock-unresolved", "AWS::S3::Bucket { Properties exists }", json.dumps({"Resources": "x"})),
    ("float-inf", "a == 5", '{"a": 1e400}'),                                  # path_value.rs:496-507
]


def _oracle_error(fn):
    try:
        fn()
    except GuardError as e:
        return FFI_CODES.get(e.kind, -1), e.display()
    raise AssertionError("the oracle did not abort")


@pytest.mark.parametrize("name,rules,data", ABORTS, ids=[a[0] for a in ABORTS])
def test_validate_abort_code_and_message_vs_oracle(name, rules, data):
    R, D = [("r.guard", rules)], [("d.json", data)]
    for fmt in ("json", "yaml", "sarif") if name == "float-inf" else ("json", "yaml", "sarif", "junit"):
        code, msg = _oracle_error(lambda: oracle_validate(R, D, output=fmt, raise_errors=True))
        with pytest.raises(guard_amd.GuardError) as ei:
            guard_amd.validate_structured(R, D, output=fmt)
        assert (ei.value.code, ei.value.message) == (code, msg), fmt


@pytest.mark.parametrize("name,rules,data", ABORTS, ids=[a[0] for a in ABORTS])
def test_run_checks_abort_code_and_message_vs_oracle(name, rules, data):
    code, msg = _oracle_error(lambda: oracle_run_checks(data, "d.json", rules, "r.guard"))
    with pytest.raises(guard_amd.GuardError) as ei:
        guard_amd.run_checks(data, "d.json", rules, "r.guard")
    assert (ei.value.code, ei.value.message) == (code, msg)


def test_junit_keeps_parse_error_exit_code_over_fail():
    """one unparsable rules file + one FAILing rule: 19 for json/yaml/sarif, 5 for junit"""
    rules = [("bad.guard", "rule r { missing_rule }"), ("fail.guard", "Resources.*.Properties.Port == 1")]
    data = [("d.json", DOC)]
    for fmt, want in (("json", 19), ("yaml", 19), ("sarif", 19), ("junit", 5)):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert ecode == want
        assert (code, out) == (ecode, exp), fmt


def test_test_command_rules_parse_error_and_empty_rules():
    """`cfn-guard test` with an unparsable rules file writes the reference's error report and exits 1
    in text mode (test.rs:300-303), 0 in the structured formats (test.rs:338-350); a rules file with no rules writes nothing and exits 0"""
    from guard_oracle.testcmd import run_test as oracle_test
    spec = ("spec.yaml", "- input: {}\n  expectations:\n    rules:\n      r: PASS\n")
    for rules in ("rule r { missing_rule }", "# only a comment\n", "rule r {\n  Resources.x == << m >>\n}\n"):
        for fmt in ("text", "json", "yaml", "junit"):
            exp, ecode = oracle_test(rules, "r.guard", [spec], fmt)
            got, code = guard_amd.run_test(rules, "r.guard", [spec], fmt)
            assert (code, got) == (ecode, exp), (rules, fmt)
            # text: TEST_ERROR_STATUS_CODE; structured: exit_code stays SUCCESS (test.rs:338-350)
            assert code == (0 if rules.startswith("#") or fmt != "text" else 1)


def test_test_command_invalid_rule_golden():
    """guard/tests/test_command.rs:183-200: the test command on an unparsable rules file prints the
    nom error verbatim (position, context, fragment) and exits 1"""
    import os
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "parse_error_cases.json"), encoding="utf-8"))
    case = [c for c in cases if c["src"] == "test_command.rs:193"][0]
    spec = ("test.yaml", "- input: {}\n  expectations:\n    rules:\n      r: PASS\n")
    got, code = guard_amd.run_test(case["text"], case["file"], [spec], "text")
    assert (code, got) == (1, "Parse Error on ruleset file " + case["expected"] + "\n")
