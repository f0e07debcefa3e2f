"""guard-ffi run_checks(verbose = true) on the GPU: the pretty serde EventRecord tree
(commands/helper.rs:62-64; RecordType / ClauseCheck serde shapes, rules/mod.rs:165-355).

The verbose kernel (eval_core.inc GG_VERBOSE) records every event in evaluation order and the host
rebuilds the tree (reporter.cpp verbose_tree).  Pinned against the reference's one golden
(guard/tests/functional.rs:7-160) and byte-compared with the oracle's tree (RecordTracker,
eval_context.rs:999-1060) over rule sets that open every container kind: file, rule and its
condition, type blocks with conditions and per-value blocks, when blocks, block clauses with
missing values, named and parameterized rules, disjunctions of the three clause types, map and
list filters, map-key filters, unary / empty / IN / not-comparable checks and count().
The Disjunction context (`type_name::<T>()`) is not pinned by any reference test; it follows the
crate layout (cfn_guard::rules::exprs) -- "parity unpinned" for that string only.
"""
import json
import os

import pytest

import guard_amd
import synth
from guard_oracle import run_checks as oracle_run_checks
from guard_oracle.errors import GuardError as OracleGuardError
from rulepack import rule_pack

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")

EVENT_RULES = r"""
let buckets = Resources.*[ Type == 'AWS::S3::Bucket' ]
let lit = 5
let names = Resources.*[ Type == 'AWS::S3::Bucket' or Type == 'AWS::EC2::Volume' ].Properties.Name

rule named_ok { Resources exists }
rule uses_named when named_ok { %buckets.Properties.Name exists <<name needed>> }
rule not_named { not named_ok or Resources.x exists }
rule types when %buckets !empty {
  AWS::S3::Bucket when Properties.Name exists {
    Properties.Name == /^b/ or Properties.Name IN ['x', 'y']
    Properties.Tags[*] { Key exists  Value != 'bad' }
  }
  AWS::EC2::Volume { Properties.Size <= 256 }
}
rule blocks {
  Resources.*[ Type == 'AWS::EC2::Volume' ] {
    Properties.Missing.Deep exists
  }
  Resources.* { Type is_string }
  when Resources exists { %lit == 5 }
}
rule check_param(x) { %x exists }
rule calls { check_param(Resources) <<param msg>> }
rule keys_filter { Resources[ keys == /^b/ ] !empty  Resources[ keys IN ['a', 'b1'] ] exists }
rule counts { let c = count(Resources.*)  %c > 1 }
rule list_filter { Resources.*.Properties.Tags[ Key == 'env' ].Value == 'prod' }
rule empty_check { Resources.*[ Type == 'Nope' ] empty }
rule notcmp { Resources.*.Properties.Size > 'abc' }
rule queryin { Resources.*.Properties.Name IN %names }
rule some_vals { some Resources.*.Properties.Tags[*].Value == 'prod' }
rule skipped when Resources.nothing exists { Resources exists }
rule guard_when {
  Resources.*[ Type == 'AWS::S3::Bucket' ] {
    when Properties.Name exists or Properties.Other exists { Properties.Name is_string }
  }
  Resources.*.Properties.Missing { Deep exists }
}
"""

EVENT_DOCS = [
    {"Resources": {
        "b1": {"Type": "AWS::S3::Bucket", "Properties": {"Name": "bucket-one", "Tags": [
            {"Key": "env", "Value": "prod"}, {"Key": "team", "Value": "bad"}]}},
        "v1": {"Type": "AWS::EC2::Volume", "Properties": {"Size": 300, "Name": "x"}},
        "v2": {"Type": "AWS::EC2::Volume", "Properties": {"Size": 100, "Missing": {"Deep": 1}}}}},
    {"Resources": {
        "a": {"Type": "AWS::S3::Bucket", "Properties": {"Name": "zeta", "Tags": []}},
        "other": {"Type": 5, "Properties": {"Size": "big"}}}},
    {"Resources": {}},
    {"Parameters": {"p": 1}},
]


def _oracle(data, dname, rules, rname):
    try:
        return oracle_run_checks(data, dname, rules, rname, verbose=True), None
    except OracleGuardError as e:
        return None, e


def _check(data, dname, rules, rname):
    exp, oerr = _oracle(data, dname, rules, rname)
    if oerr is not None:
        with pytest.raises(guard_amd.GuardError):
            guard_amd.run_checks(data, dname, rules, rname, verbose=True)
        return False
    got = guard_amd.run_checks(data, dname, rules, rname, verbose=True)
    assert got == exp, (rname, dname)
    return True


def test_verbose_functional_golden():
    """guard/tests/functional.rs:7-160 -- compared as parsed JSON, as that test does, and as text
    with the oracle"""
    c = json.load(open(os.path.join(G, "verbose_golden.json")))[0]
    got = guard_amd.run_checks(c["data"], c["data_name"], c["rules"], c["rules_name"], verbose=True)
    assert json.loads(got) == c["expected"]
    assert got == oracle_run_checks(c["data"], c["data_name"], c["rules"], c["rules_name"], verbose=True)


def test_verbose_every_event_kind_vs_oracle():
    ran = 0
    for i, d in enumerate(EVENT_DOCS):
        ran += _check(json.dumps(d), "ev%d.json" % i, EVENT_RULES, "events.guard")
    assert ran == len(EVENT_DOCS)


def test_verbose_rule_pack_vs_oracle():
    """the cfg-2 rule pack (reference rule files) over synthetic CloudFormation templates"""
    docs = synth.cfn_corpus(3, start=2000, n_resources=10)
    ran = 0
    for name, text in rule_pack():
        for i, d in enumerate(docs):
            ran += _check(d, "doc%d.json" % i, text, name)
    assert ran > 0


def test_verbose_reference_specs_vs_oracle():
    """the reference's own test specs (rules x input cases, tests/golden/expectations.json)"""
    cases = json.load(open(os.path.join(G, "expectations.json")))
    ran = 0
    for c in cases:
        ran += _check(c["input_json"], "input-%d.json" % c["case"], c["rules_text"], c["rules_name"])
    assert ran > len(cases) // 2


def _docs(kind):
    if kind == "tf":
        return synth.tf_corpus(2, start=500, n_resources=15)
    if kind == "config":
        return synth.config_corpus(2, start=600)
    return synth.cfn_corpus(2, start=400, n_resources=12)


@pytest.mark.parametrize("pack,kind", [("edge_rulepack", "cfn"), ("capture_rulepack", "cfn"), ("conv_rulepack", "cfn"),
                                       ("cfg3_rulepack", "cfn"), ("tf_rulepack", "tf"), ("net_rulepack", "config")])
def test_verbose_local_packs_vs_oracle(pack, kind):
    p = os.path.join(G, pack)
    rules = [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
    ran = 0
    for name, text in rules:
        for i, d in enumerate(_docs(kind)):
            ran += _check(d, "doc%d.json" % i, text, name)
    assert ran > 0
