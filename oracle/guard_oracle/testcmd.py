"""``cfn-guard test`` restatement (TEST INFRASTRUCTURE ONLY -- the parity oracle).

Follows ``commands/test.rs`` (spec files: ``Vec<TestSpec>`` via serde_yaml, then serde_json,
:480-484), ``reporters/test/mod.rs`` (get_by_rules / get_status_result), the text reporter
``reporters/test/generic.rs`` and the structured reporter ``reporters/test/structured.rs`` with
``handle_structured_single_report`` (test.rs:326-380).  One rules file x spec files.

get_by_rules groups the rule records in a Rust ``HashMap``, whose iteration order is random per
process, so the reference's order of rules *within one test case* is unspecified; this restatement
uses the rules' first appearance in the file.  The reference's goldens (one rule per file) pin the
rest byte for byte.
"""
from .errors import GuardError
from . import evaluator as E
from .formats import _xml_escape, to_yaml
from .loader import load_serde_yaml_tree, serde_tree_to_pv, load_serde_json
from .parser import parse_rules
from .pv import LIST, MAP, STRING
from .report import OMap, to_json_pretty

TEST_ERROR, TEST_FAILURE, SUCCESS = 1, 7, 0


def _load_specs(text, path):
    try:
        spec = serde_tree_to_pv(load_serde_yaml_tree(text))
    except Exception:
        try:
            spec = load_serde_json(text)
        except Exception as e:
            raise GuardError("ParseError", "Unable to process data in file %s, Error %s," % (path, e))
    if spec.kind != LIST:
        raise GuardError("ParseError", "Unable to process data in file %s, Error invalid type" % path)
    out = []
    for case in spec.val:
        if case.kind != MAP:
            raise GuardError("ParseError", "Unable to process data in file %s, Error invalid type" % path)
        vals = case.val.values
        name = vals.get("name")
        exp = vals.get("expectations")
        if "input" not in vals or exp is None or exp.kind != MAP or exp.val.values.get("rules") is None:
            raise GuardError("ParseError", "Unable to process data in file %s, Error missing field" % path)
        rules = exp.val.values["rules"]
        expected = [(k, v.val) for k, v in rules.val.values.items()] if rules.kind == MAP else []
        out.append((None if name is None or name.kind != STRING else name.val, vals["input"], expected))
    return out


def _status(s):
    if s not in ("PASS", "FAIL", "SKIP"):
        raise GuardError("ParseError", "Unable to parse status {}".format(s))
    return s


def _by_rules(rf, inp):
    root = E.RootScope(rf, inp)
    E.eval_rules_file(rf, root, None)
    by = {}
    for ch in root.recorder.final_event.children:
        if ch.container and ch.container[0] == "RuleCheck":
            by.setdefault(ch.container[1], []).append(ch.container[2])
    return by


def get_status_result(expected, got):
    """reporters/test/mod.rs:20-54 -> (matched status or None, statuses seen before the match)"""
    statuses, all_skipped = [], 0
    for g in got:
        if expected == "SKIP":
            if g == "SKIP":
                all_skipped += 1
        elif g == expected:
            return expected, statuses
        statuses.append(g)
    if expected == "SKIP" and all_skipped == len(got):
        return expected, statuses
    return None, statuses


def run_test(rules_text, rules_name, specs, output="text"):
    """specs: [(path, text)].  Returns (stdout text, exit code)."""
    try:
        rf = parse_rules(rules_text, rules_name)
    except GuardError as e:
        # test.rs:300-303 (plain text): TEST_ERROR_STATUS_CODE; 345-350 (structured TestResult::Err):
        # handle_structured_single_report's exit_code stays SUCCESS_STATUS_CODE on this branch
        if output == "text":
            return "Parse Error on ruleset file %s\n" % e.display(), TEST_ERROR
        return _structured_error(rules_name, e.display(), output, SUCCESS)
    if rf is None:
        # Ok(None): nothing written, SUCCESS_STATUS_CODE (test.rs:315, 366)
        return "", SUCCESS
    if output == "text":
        return _generic(rf, specs)
    return _structured(rf, rules_name, specs, output)


def _generic(rf, specs):
    out, code, counter = [], SUCCESS, 1
    for path, text in specs:
        try:
            cases = _load_specs(text, path)
        except GuardError as e:
            out.append("Error processing %s\n" % e.display())
            code = TEST_ERROR
            continue
        for name, inp, expected in cases:
            out.append("Test Case #%d\n" % counter)
            if name is not None:
                out.append("Name: %s\n" % name)
            exp = dict(expected)
            by = _by_rules(rf, inp)
            res = {}
            for rule, got in by.items():
                if rule not in exp:
                    out.append("  No Test expectation was set for Rule %s\n" % rule)
                    continue
                e = _status(exp[rule])
                m, st = get_status_result(e, got)
                if m is not None:
                    res.setdefault("PASS", []).append("%s: Expected = %s" % (rule, m))
                else:
                    res.setdefault("FAIL", []).append("%s: Expected = %s, Evaluated = [%s]" % (rule, e, ", ".join(st)))
            if "FAIL" in res:
                code = TEST_FAILURE
            for k in sorted(res):
                out.append("  %s Rules:\n" % k)
                for line in dict.fromkeys(res[k]):
                    out.append("    %s\n" % line)
            out.append("\n")
            counter += 1
    return "".join(out), code


def _structured(rf, rules_name, specs, output):
    cases_out, junit_cases, failures, code = [], [], 0, SUCCESS
    for path, text in specs:
        try:
            cases = _load_specs(text, path)
        except GuardError as e:
            return _structured_error(rules_name, e.display(), output)
        for name, inp, expected in cases:
            exp = dict(expected)
            by = _by_rules(rf, inp)
            passed, failed, skipped = [], [], []
            for rule, got in by.items():
                if rule not in exp:
                    skipped.append(OMap([("name", rule)]))
                    continue
                e = _status(exp[rule])
                m, st = get_status_result(e, got)
                if m is not None:
                    passed.append(OMap([("name", rule), ("evaluated", m)]))
                else:
                    failed.append(OMap([("name", rule), ("expected", e), ("evaluated", st)]))
            tname = name or ""
            for p in passed:
                junit_cases.append((tname, p.items[0][1], None))
            for f in failed:
                junit_cases.append((tname, f.items[0][1], "Expected = %s, Evaluated = [%s]" % (f.items[1][1], ", ".join(f.items[2][1]))))
            failures += len(failed)
            if failed:
                code = TEST_FAILURE
            cases_out.append(OMap([("name", tname), ("passed_rules", passed), ("failed_rules", failed),
                                   ("skipped_rules", skipped)]))
    result = OMap([("rule_file", rules_name), ("test_cases", cases_out)])
    if output == "json":
        return to_json_pretty(result), code
    if output == "yaml":
        return to_yaml(result), code
    lines = ['<?xml version="1.0" encoding="UTF-8"?>',
             '<testsuites name="cfn-guard test report" tests="%d" failures="%d" errors="0" time="0">' % (len(junit_cases), failures),
             '    <testsuite name="%s" errors="0" failures="%d" time="0">' % (_xml_escape(rules_name), failures)]
    for tid, rname, msg in junit_cases:
        if msg is None:
            lines.append('        <testcase id="%s" name="%s" time="0" status="pass"/>' % (_xml_escape(tid), _xml_escape(rname)))
        else:
            lines.append('        <testcase id="%s" name="%s" time="0">' % (_xml_escape(tid), _xml_escape(rname)))
            lines.append('            <failure>%s</failure>' % _xml_escape(msg))
            lines.append('        </testcase>')
    lines += ['    </testsuite>', '</testsuites>']
    return "\n".join(lines) + "\n", code


def _structured_error(rules_name, error, output, code=TEST_ERROR):
    """TestResult::Err report; `code`: TEST_ERROR for a spec file that does not load (structured.rs:57-59
    get_exit_code), SUCCESS for an unparsable rules file (test.rs:338-350)"""
    result = OMap([("rule_file", rules_name), ("error", error)])
    if output == "json":
        return to_json_pretty(result), code
    if output == "yaml":
        return to_yaml(result), code
    return ("\n".join(['<?xml version="1.0" encoding="UTF-8"?>',
                       '<testsuites name="cfn-guard test report" tests="1" failures="0" errors="1" time="0">',
                       '    <testsuite name="%s" errors="1" failures="0" time="0">' % _xml_escape(rules_name),
                       '        <testcase name="%s" time="0" status="error">' % _xml_escape(rules_name),
                       '            <error>%s</error>' % _xml_escape(error),
                       '        </testcase>', '    </testsuite>', '</testsuites>']) + "\n", code)
