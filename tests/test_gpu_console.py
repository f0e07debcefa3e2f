"""GPU parity of `cfn-guard validate` without --structured (the console reporters: summary table,
CFN / Terraform / generic single-line summaries, -o json / yaml per pair, --verbose, --print-json),
through the C ABI (cfn_guard_validate_console):

* the reference's own goldens (guard/tests/validate.rs:237-345, 405-418, 488-540 with
  resources/validate/output-dir/*.out) -- byte-identical stdout and exit codes;
* the cases whose rules need fancy-regex look-behind (outside the DFA subset): an explicit
  "unsupported on MI355X path" abort, nothing reported for the pair;
* rule packs x synthetic corpora in every output mode against the oracle's restatement
  (oracle/guard_oracle/console.py), which is pinned by the same goldens.
"""
import os

import pytest

import console_cases
import guard_amd
import rulepack
import synth
from guard_oracle.console import validate_console as oracle_console

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
CASES = console_cases.cases()


@pytest.mark.parametrize("case", [c for c in CASES if not c[6]], ids=[c[0] for c in CASES if not c[6]])
def test_console_golden_on_gpu(case):
    name, rules, data, opts, expected, code, _ = case
    out, rc, err = guard_amd.validate_console(rules, data, **opts)
    assert (rc, err) == (code, "")
    # cases the reference pins by exit code only: the oracle's restatement fixes the text
    assert out == (expected if expected is not None else oracle_console(rules, data, **opts)[0])


def test_console_payload_type_block_error():
    rules, data = console_cases._payload(console_cases.PAYLOAD_TYPE_BLOCK)
    exp = oracle_console(rules, data)
    got = guard_amd.validate_console(rules, data)
    assert got == exp


FN_OUT_OF_SCOPE = ["complex_rules.guard", "converters.guard", "failing_complex_rule.guard", "join.guard",
                   "join_with_message.guard", "json_parse.guard", "now.guard", "parse_epoch.guard",
                   "regex_replace.guard", "string_manipulation.guard", "substring.guard", "url_decode.guard"]


@pytest.mark.parametrize("rule", FN_OUT_OF_SCOPE)
def test_console_builtin_functions_are_explicitly_unsupported(rule):
    """validate.rs:709-785 with a built-in other than count() (out of scope): the MI355X
    path refuses the rules file loudly instead of evaluating it some other way"""
    out, rc, err = guard_amd.validate_console(console_cases._fn_rules(rule), console_cases._fn_data(),
                                              summary=("all",), verbose=True)
    assert rc == -1 and out == ""
    assert "unsupported on MI355X path" in err


@pytest.mark.parametrize("case", [c for c in CASES if c[6]], ids=[c[0] for c in CASES if c[6]])
def test_console_lookaround_is_explicitly_unsupported(case):
    name, rules, data, opts, expected, code, _ = case
    out, rc, err = guard_amd.validate_console(rules, data, **opts)
    assert rc == -1
    assert "unsupported on MI355X path" in err
    # the first pair evaluated is a look-behind rules file: nothing is printed before the abort
    assert out == ""


def _pack(d):
    p = os.path.join(G, d)
    return [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]


PACKS = {
    "cfg2": lambda: (rulepack.rule_pack("cfg2"), [("t-%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(3, start=0))]),
    "tf": lambda: (_pack("tf_rulepack"), [("plan-%d.json" % i, d) for i, d in enumerate(synth.tf_corpus(3, start=0, n_resources=10))]),
    "net": lambda: (_pack("net_rulepack"), [("s-%d.json" % i, d) for i, d in enumerate(synth.config_corpus(2, start=0))]),
    "ops": lambda: (_pack("ops_rulepack"), [("t-%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(2, start=5))]),
    "edge": lambda: (_pack("edge_rulepack"), [("t-%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(2, start=7))]),
    "capture": lambda: (_pack("capture_rulepack"), [("t-%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(1, start=9))]),
    "validate": lambda: ([r for r in console_cases._rules(*["rules-dir/" + f for f in console_cases._dir("rules-dir", (".guard",))])
                          if "lookbehind" not in r[0]],
                         console_cases._data(*["data-dir/" + f for f in console_cases._dir("data-dir", (".yaml",))])),
}
OPTS = [
    {"summary": ("all",)},
    {"summary": ("fail",), "verbose": True, "print_json": True},
    {"summary": ("pass", "skip")},
    {"summary": ("none",)},
    {"output": "json"},
    {"output": "yaml", "summary": ("all",), "verbose": True},
]


@pytest.mark.parametrize("pack", sorted(PACKS))
def test_console_packs_vs_oracle(pack):
    rules, data = PACKS[pack]()
    for opts in OPTS:
        exp = oracle_console(rules, data, **opts)
        got = guard_amd.validate_console(rules, data, **opts)
        assert got[1:] == exp[1:], (pack, opts)
        assert got[0] == exp[0], (pack, opts)


def _console_pack():
    d = os.path.join(G, "console_rulepack")
    rules = _pack("console_rulepack")
    data = [(f, open(os.path.join(d, f)).read()) for f in ("cdk_template.yaml", "tf_plan.json", "plain.json")]
    return rules, data


def test_console_branches_vs_oracle():
    """tests/golden/console_rulepack reaches every reporter branch: CFN resources with CDK paths and code
    snippets (unary / binary / IN / unresolved / block / disjunction / `some` / parameterized rules with
    messages), a Terraform plan's resource_changes (TfAware), generic data (dependent rules, a block whose
    query cannot resolve)"""
    rules, data = _console_pack()
    for opts in OPTS + [{"summary": ("all",), "print_json": True}]:
        exp = oracle_console(rules, data, **opts)
        got = guard_amd.validate_console(rules, data, **opts)
        assert got == exp, opts


def test_console_terraform_unresolved_panics_like_the_reference():
    """tf.rs single_line: a failing value that stops at .../change/after does not match
    RESOURCE_CHANGE_EXTRACTION -> unreachable!(): the run aborts with the panic text"""
    rules = [("tf_unresolved.guard", open(os.path.join(G, "console_rulepack", "tf_unresolved.guard.txt")).read())]
    _, data = _console_pack()
    exp = oracle_console(rules, data[1:2])
    got = guard_amd.validate_console(rules, data[1:2])
    assert exp[1] == got[1] == -1
    assert "internal error: entered unreachable code" in exp[2] and "internal error: entered unreachable code" in got[2]
    assert got[0] == exp[0]


def test_console_parse_error_and_params():
    rules = [("bad.guard", "rule {"), ("db_param_port_rule.guard",
                                        open(os.path.join(G, "params", "db_param_port_rule.guard")).read())]
    pdir = os.path.join(G, "params")
    data = [("db_resource.yaml", open(os.path.join(pdir, "db_resource.yaml")).read())]
    idir = os.path.join(pdir, "input-parameters-dir")
    params = [(f, open(os.path.join(idir, f)).read()) for f in sorted(os.listdir(idir))]
    for opts in ({"summary": ("all",)}, {"output": "json"}):
        exp = oracle_console(rules, data, params=params, **opts)
        got = guard_amd.validate_console(rules, data, params=params, **opts)
        assert got == exp
