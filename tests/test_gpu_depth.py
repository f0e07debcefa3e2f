"""Evaluation depth against the device lane stack.

The reference evaluates rule references, nested blocks and `when` blocks recursively on the host stack
(eval.rs:1227-1289 eval_guard_named_clause, 1303-1426 eval_guard_block_clause, 1837-1906 eval_rule); the
device evaluator recurses too, in a 16 KB dynamic lane stack, and checks its stack pointer where it recurses
(eval_core.inc stack_low).  A chain up to the guard evaluates byte-equal to the oracle; one level past it ends
the run with the explicit "evaluation depth limit exceeded" error (never a fault), in lane and wave mode.
The deepest passing chain is found by bisection on the GPU and pinned on both sides."""
import json

import pytest

import guard_amd
from guard_oracle import validate_structured as oracle_validate

pytestmark = pytest.mark.gpu

DOC = json.dumps({"Resources": {"b": {"Type": "AWS::S3::Bucket", "Properties": {"Name": "x"}}}})


def named_chain(n):
    # evaluated first, the deepest rule references the next one down: n rule levels (eval_rule ->
    # eval_conj -> named clause -> rule_status -> eval_rule ...); rule_status memoizes only references
    lines = ["rule r%d {\n    r%d\n}" % (k, k - 1) for k in range(n, 0, -1)]
    lines.append("rule r0 { Resources.*.Properties.Name == 'y' }")
    return "\n".join(lines) + "\n"


def block_chain(n):
    # n nested block clauses, each selecting `a` from the previous level's value (ValueScope), over a
    # document nested as deep: {"a": {"a": ... {"v": "x"}}}
    body = "v == 'y'"
    for _ in range(n):
        body = "a { %s }" % body
    return "rule deep { %s }\n" % body


def _doc(chain, n):
    if chain is block_chain:
        d = {"v": "x"}
        for _ in range(n):
            d = {"a": d}
        return json.dumps(d)
    return DOC


def when_chain(n):
    body = "Resources.*.Properties.Name == 'y'"
    for _ in range(n):
        body = "when Resources exists { %s }" % body
    return "rule deep { %s }\n" % body


def param_chain(n):
    # parameterized rules calling each other (eval_parameterized_rule_call, eval.rs:1574-1618)
    lines = ["rule p0(v) { %v == 'y' }"]
    for k in range(1, n + 1):
        lines.append("rule p%d(v) { p%d(%%v) }" % (k, k - 1))
    lines.append("rule top { p%d(Resources.*.Properties.Name) }" % n)
    return "\n".join(lines) + "\n"


def _run(chain, n, mode):
    s = guard_amd.Session()
    try:
        s.configure(mode, 0)
        s.add_rules(chain(n), "deep.guard")
        s.add_docs([_doc(chain, n)], ["d.json"])
        s.eval(1)
        return s.report()
    finally:
        s.close()


def _passes(chain, n, mode):
    try:
        _run(chain, n, mode)
        return True
    except guard_amd.GuardError as e:
        assert e.code == -1 and "evaluation depth limit exceeded" in e.message, (e.code, e.message)
        return False


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("chain", [named_chain, block_chain, when_chain, param_chain])
def test_depth_limit_and_one_past(chain, mode):
    lo, hi = 1, 256   # lo passes, hi does not
    assert _passes(chain, lo, mode)
    assert not _passes(chain, hi, mode)   # far past the stack: the explicit error, not a fault
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if _passes(chain, mid, mode):
            lo = mid
        else:
            hi = mid
    # at the limit: the reference's bytes; one past it: the error (checked by _passes)
    rules = [("deep.guard", chain(lo))]
    exp, ecode, _ = oracle_validate(rules, [("d.json", _doc(chain, lo))])
    assert _run(chain, lo, mode) == (exp, ecode)
    assert hi == lo + 1
    # the guard leaves realistic nesting far inside the stack
    assert lo >= 12, lo


def test_depth_error_through_the_c_abi():
    """the explicit error through the one-string entry (the FFI's panic code -1, the message named)"""
    with pytest.raises(guard_amd.GuardError) as g:
        guard_amd.validate_structured([("deep.guard", named_chain(400))], [("d.json", DOC)])
    assert g.value.code == -1 and "evaluation depth limit exceeded" in g.value.message
