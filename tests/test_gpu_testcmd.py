"""`cfn-guard test` on the MI355X path (C ABI cfn_guard_test) against the reference's goldens
(guard/tests/test_command.rs:157-178, 263-290) and the oracle (oracle/guard_oracle/testcmd.py)."""
import json
import os

import pytest

import guard_amd
from guard_oracle.testcmd import run_test as oracle_test

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
T = os.path.join(G, "test-command")
RN = "resources/validate/rules-dir/s3_bucket_server_side_encryption_enabled.guard"


def _rules():
    return open(os.path.join(G, "validate", "rules-dir", "s3_bucket_server_side_encryption_enabled.guard")).read()


@pytest.mark.parametrize("fmt,gold,spec", [
    ("text", "test_data_file.out", "json"), ("text", "test_data_file.out", "yaml"),
    ("json", "structured_single_report_json.out", "yaml"), ("yaml", "structured_single_report_yaml.out", "yaml"),
    ("junit", "structured_single_report_junit.out", "yaml")])
def test_test_command_goldens(fmt, gold, spec):
    sp = "s3_bucket_server_side_encryption_enabled." + spec
    out, code = guard_amd.run_test(_rules(), RN, [("resources/test-command/data-dir/" + sp, open(os.path.join(T, sp)).read())], fmt)
    assert code == 0
    assert out == open(os.path.join(T, gold)).read()


def test_reference_example_specs_vs_oracle():
    """every reference spec in tests/golden/expectations.json, regrouped per (rules file, spec): one
    `test` run each, all formats, against the oracle"""
    cases = json.load(open(os.path.join(G, "expectations.json")))
    groups = {}
    for c in cases:
        groups.setdefault((c["rules_name"], c["spec"]), (c["rules_text"], []))[1].append(c)
    for (rname, spec), (rtext, cs) in sorted(groups.items()):
        spec_json = json.dumps([{"name": "case %d" % c["case"], "input": json.loads(c["input_json"]),
                                 "expectations": {"rules": c["expected"]}} for c in cs])
        for fmt in ("text", "json", "yaml", "junit"):
            exp = oracle_test(rtext, rname, [(spec, spec_json)], fmt)
            got = guard_amd.run_test(rtext, rname, [(spec, spec_json)], fmt)
            assert got == exp, (rname, spec, fmt)


def test_test_command_directory_and_shorthand_goldens():
    """cfn_guard_test_dir: guard/tests/test_command.rs:297-313 (the dir's rules files with their tests,
    structured_directory_report_{json,yaml,junit}.out) and cfn_guard_test on :135-150 (shorthand:
    expectations for another rule, test_data_file_with_shorthand_reference.out); exit 0"""
    from test_oracle_golden import directory_pairs
    for fmt in ("json", "yaml", "junit"):
        out, code = guard_amd.run_test_dir(directory_pairs(), fmt)
        assert code == 0 and out == open(os.path.join(T, "structured_directory_report_%s.out" % fmt)).read(), fmt
    for sp in ("json", "yaml"):
        spec = "s3_bucket_logging_enabled_tests." + sp
        out, code = guard_amd.run_test(_rules(), RN, [("resources/test-command/data-dir/" + spec, open(os.path.join(T, spec)).read())])
        assert code == 0 and out == open(os.path.join(T, "test_data_file_with_shorthand_reference.out")).read(), sp


def test_test_command_directory_vs_oracle():
    """directory mode in every format against the oracle, with a rules file without tests, an
    unparsable rules file (TEST_ERROR in structured mode, TEST_FAILURE in text mode, test.rs:255-259,
    416-423), a rules file with no rules and a failing expectation"""
    from guard_oracle.testcmd import run_test_dir as oracle_dir
    from test_oracle_golden import directory_pairs
    pairs = directory_pairs()
    spec = pairs[0][2]
    extra = [("none.guard", "rule r { Resources exists }", []),
             ("bad.guard", "rule r { Resources.x == << m >>\n}", spec),
             ("empty.guard", "# nothing\n", spec),
             ("fails.guard", "rule S3_BUCKET_LOGGING_ENABLED { Resources.* exists }", spec)]
    for combo in (pairs, pairs + extra, extra[::-1] + pairs):
        for fmt in ("text", "json", "yaml", "junit"):
            assert guard_amd.run_test_dir(combo, fmt) == oracle_dir(combo, fmt), ([c[0] for c in combo], fmt)


def test_test_command_verbose_goldens():
    """cfn_guard_test_ex / cfn_guard_test_dir with verbose: the verbose wave kernel's event stream drawn
    as print_verbose_tree (test_command.rs:223-257 goldens); structured formats refuse the flag (18)"""
    from test_oracle_golden import directory_pairs
    for sp in ("json", "yaml"):
        spec = "s3_bucket_server_side_encryption_enabled." + sp
        out, code = guard_amd.run_test(_rules(), RN, [("resources/test-command/data-dir/" + spec, open(os.path.join(T, spec)).read())],
                                       "text", verbose=True)
        assert code == 0 and out == open(os.path.join(T, "test_data_file_verbose.out")).read(), sp
    out, code = guard_amd.run_test_dir(directory_pairs(), "text", verbose=True)
    assert code == 0 and out == open(os.path.join(T, "test_data_dir_verbose.out")).read()
    with pytest.raises(guard_amd.GuardError) as ei:
        guard_amd.run_test(_rules(), RN, [("s.yaml", "[]")], "json", verbose=True)
    assert ei.value.code == 18


def test_test_command_verbose_vs_oracle():
    """every reference example spec (tests/golden/expectations.json) through `test --verbose`: the text
    EventRecord trees (every container and value-check kind the packs reach) equal the oracle's"""
    cases = json.load(open(os.path.join(G, "expectations.json")))
    groups = {}
    for c in cases:
        groups.setdefault((c["rules_name"], c["spec"]), (c["rules_text"], []))[1].append(c)
    for (rname, spec), (rtext, cs) in sorted(groups.items()):
        spec_json = json.dumps([{"name": "case %d" % c["case"], "input": json.loads(c["input_json"]),
                                 "expectations": {"rules": c["expected"]}} for c in cs])
        exp = oracle_test(rtext, rname, [(spec, spec_json)], "text", verbose=True)
        got = guard_amd.run_test(rtext, rname, [(spec, spec_json)], "text", verbose=True)
        assert got == exp, (rname, spec)
