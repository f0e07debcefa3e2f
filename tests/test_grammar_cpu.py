"""Grammar pinning (no GPU): the rule texts of the reference's parser unit tests
(guard/src/rules/parser_tests.rs), lifted to whole rules files by tests/golden/make_grammar_cases.py,
must be accepted / rejected as those tests assert -- by the product's parser (csrc/rules_parser.cpp,
through gg_parse_rules) and by the oracle's (oracle/guard_oracle/parser.py) independently, so a
misreading shared by both restatements shows up against the reference's own expectation."""
import json
import os

import pytest

import guard_amd
from guard_oracle.errors import GuardError as OracleGuardError
from guard_oracle.parser import parse_rules as oracle_parse_rules

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "grammar_cases.json"), encoding="utf-8"))


def _native(text):
    try:
        return {0: True, 1: None}[guard_amd.parse_rules(text, "g.guard")]
    except guard_amd.GuardError as e:
        assert e.code == 5, (e.code, e.message)
        return False


def _oracle(text):
    try:
        return None if oracle_parse_rules(text, "g.guard") is None else True
    except OracleGuardError as e:
        assert e.kind == "ParseError", e
        return False


@pytest.mark.parametrize("case", CASES, ids=[c["id"] for c in CASES])
def test_grammar_case(case):
    assert _native(case["text"]) == case["accept"], ("native", case["src"], case["text"])
    assert _oracle(case["text"]) == case["accept"], ("oracle", case["src"], case["text"])
