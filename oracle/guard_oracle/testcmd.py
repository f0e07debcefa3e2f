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
from .pv import LIST, MAP, STRING, PV, MapValue
from .report import OMap, event_text, to_json_pretty

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
        # PathAwareValue::try_from(spec.input) (reporters/test/generic.rs:75): the input is its own
        # root -- paths relative to it, not to the spec file
        out.append((None if name is None or name.kind != STRING else name.val, _reroot(vals["input"], len(vals["input"].path)), expected))
    return out


def _reroot(v, cut):
    """a copy of serde-loaded value `v` with `cut` leading path characters removed (locations are 0)"""
    k = v.kind
    if k == LIST:
        return PV(LIST, v.path[cut:], 0, 0, [_reroot(e, cut) for e in v.val])
    if k == MAP:
        mv = MapValue()
        mv.keys = [PV(STRING, kp.path[cut:], 0, 0, kp.val) for kp in v.val.keys]
        mv.values = {key: _reroot(e, cut) for key, e in v.val.values.items()}
        return PV(MAP, v.path[cut:], 0, 0, mv)
    return PV(k, v.path[cut:], 0, 0, v.val)


def _status(s):
    if s not in ("PASS", "FAIL", "SKIP"):
        raise GuardError("ParseError", "Unable to parse status {}".format(s))
    return s


def _by_rules(rf, inp, tree=None):
    root = E.RootScope(rf, inp)
    E.eval_rules_file(rf, root, None)
    if tree is not None:
        tree.append(root.recorder.final_event)
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


def run_test(rules_text, rules_name, specs, output="text", verbose=False):
    """specs: [(path, text)].  Returns (stdout text, exit code).  verbose: each test case's
    EventRecord tree as text (reporters/test/generic.rs:116-118); with a structured output the
    reference refuses the flags (test.rs:134-137, IllegalArguments)."""
    if verbose and output != "text":
        raise GuardError("IllegalArguments", "Cannot provide an output_type of JSON, YAML, or JUnit while the verbose flag is set")
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
        return _generic(rf, specs, verbose)
    return _structured(rf, rules_name, specs, output)


def _generic(rf, specs, verbose=False):
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
            tree = []
            by = _by_rules(rf, inp, tree)
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
            if verbose:
                out.append(event_text(tree[0]))
            if "FAIL" in res:
                code = TEST_FAILURE
            for k in sorted(res):
                out.append("  %s Rules:\n" % k)
                for line in dict.fromkeys(res[k]):
                    out.append("    %s\n" % line)
            out.append("\n")
            counter += 1
    return "".join(out), code


def _result(rf, rules_name, specs):
    """One TestResult (reporters/test/structured.rs:33-67): StructuredTestReporter::evaluate returns
    Err at the first spec file that does not load.  Returns (serde object, exit code, JUnit suite)."""
    cases_out, junit_cases, failures, code = [], [], 0, SUCCESS
    for path, text in specs:
        try:
            cases = _load_specs(text, path)
        except GuardError as e:
            return _err_result(rules_name, e.display())
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
    suite = ['    <testsuite name="%s" errors="0" failures="%d" time="0">' % (_xml_escape(rules_name), failures)]
    for tid, rname, msg in junit_cases:
        if msg is None:
            suite.append('        <testcase id="%s" name="%s" time="0" status="pass"/>' % (_xml_escape(tid), _xml_escape(rname)))
        else:
            suite.append('        <testcase id="%s" name="%s" time="0">' % (_xml_escape(tid), _xml_escape(rname)))
            suite.append('            <failure>%s</failure>' % _xml_escape(msg))
            suite.append('        </testcase>')
    suite.append('    </testsuite>')
    return OMap([("rule_file", rules_name), ("test_cases", cases_out)]), code, (suite, len(junit_cases), failures, 0)


def _err_result(rules_name, error):
    """TestResult::Err (build_test_suite: one error test case)"""
    suite = ['    <testsuite name="%s" errors="1" failures="0" time="0">' % _xml_escape(rules_name),
             '        <testcase name="%s" time="0" status="error">' % _xml_escape(rules_name),
             '            <error>%s</error>' % _xml_escape(error),
             '        </testcase>', '    </testsuite>']
    return OMap([("rule_file", rules_name), ("error", error)]), TEST_ERROR, (suite, 1, 0, 1)


def _render(results, output, single):
    """serde_json pretty / serde_yaml of one TestResult or a Vec<TestResult>; JunitReport::from
    (reporters/mod.rs:35-63) sums the suites' tests, failures and errors"""
    if output == "json":
        return to_json_pretty(results[0][0] if single else [r[0] for r in results])
    if output == "yaml":
        return to_yaml(results[0][0] if single else [r[0] for r in results])
    tests = sum(r[2][1] for r in results)
    failures = sum(r[2][2] for r in results)
    errors = sum(r[2][3] for r in results)
    lines = ['<?xml version="1.0" encoding="UTF-8"?>',
             '<testsuites name="cfn-guard test report" tests="%d" failures="%d" errors="%d" time="0">' % (tests, failures, errors)]
    for r in results:
        lines += r[2][0]
    lines.append('</testsuites>')
    return "\n".join(lines) + "\n"


def _structured(rf, rules_name, specs, output):
    res = _result(rf, rules_name, specs)
    return _render([res], output, True), res[1]


def _structured_error(rules_name, error, output, code=TEST_ERROR):
    """TestResult::Err report; `code`: TEST_ERROR for a spec file that does not load (structured.rs:57-59
    get_exit_code), SUCCESS for an unparsable rules file (test.rs:338-350)"""
    return _render([_err_result(rules_name, error)], output, True), code


def _fold_code(code, test_code):
    """get_exit_code (test.rs:459-472)"""
    if code == SUCCESS:
        return test_code
    if code == TEST_ERROR:
        return code
    return TEST_ERROR if test_code == TEST_ERROR else TEST_FAILURE


def run_test_dir(pairs, output="text", verbose=False):
    """``cfn-guard test -d`` (test.rs:143-165) over [(rules_name, rules_text, [(spec_path, text)])] in the
    directory's order: handle_plaintext_directory (text, :221-283) or
    handle_structured_directory_report (:383-456).  Returns (stdout text, exit code)."""
    if verbose and output != "text":
        raise GuardError("IllegalArguments", "Cannot provide an output_type of JSON, YAML, or JUnit while the verbose flag is set")
    if output == "text":
        out, code = [], SUCCESS
        for rules_name, rules_text, specs in pairs:
            if not specs:
                out.append("Guard File %s did not have any tests associated, skipping.\n---\n" % rules_name)
                continue
            out.append("Testing Guard File %s\n" % rules_name)
            try:
                rf = parse_rules(rules_text, rules_name)
            except GuardError as e:
                out.append("Parse Error on ruleset file %s\n" % e.display())
                code = TEST_FAILURE
                out.append("---\n")
                continue
            if rf is not None:
                text, c = _generic(rf, specs, verbose)
                out.append(text)
                code = c if code == SUCCESS else code
            out.append("---\n")
        return "".join(out), code
    results, code = [], SUCCESS
    for rules_name, rules_text, specs in pairs:
        if not specs:
            continue
        try:
            rf = parse_rules(rules_text, rules_name)
        except GuardError as e:
            results.append(_err_result(rules_name, e.display()))
            code = TEST_ERROR
            continue
        if rf is None:
            continue
        res = _result(rf, rules_name, specs)
        code = _fold_code(code, res[1])
        results.append(res)
    return _render(results, output, False), code
