"""GPU parity on the other BASELINE.json workloads (configs[3], configs[4]) and on structural
equality, through the C ABI, against the CPU oracle.

* cfg 4: Terraform plan JSON (synth.tf_corpus) x tests/golden/tf_rulepack (the reference's
  terraform-infra-related/check-s3-tags-present.guard plus pack-local filter-heavy rules);
* cfg 5: AWS Config snapshots wrapped as Resources maps (synth.config_corpus) x
  tests/golden/net_rulepack (the reference's network-reachability-analysis rule plus pack-local
  regex / join rules);
* container equality (tests/golden/edge_rulepack): map / list ==, !=, IN over the iterative
  compare_eq / PartialEq.

Small batches are compared byte-for-byte with the oracle's structured JSON; full-size plans
(2000 resources, cfg 4's upper bound) are compared with the oracle on two documents and, on a
larger batch, through a size-independent property: the lane-per-tile and wave-per-tile kernels
produce identical reports.
"""
import os

import pytest

import guard_amd
import synth
from guard_oracle import validate_structured as oracle_validate

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _pack(d):
    p = os.path.join(G, d)
    return [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]


def _vs_oracle(docs, rules, prefix):
    data = [("%s-%d.json" % (prefix, i), d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    out, code = guard_amd.validate_structured(rules, data)
    assert code == ecode
    assert out == exp


def _session_report(docs, rules, mode, prefix):
    s = guard_amd.Session()
    s.configure(mode, 0)
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs(docs, ["%s-%d.json" % (prefix, i) for i in range(len(docs))])
    s.eval(1)
    assert s.stat(s.STAT["errors"]) == 0
    out, code = s.report()
    s.close()
    return out, code


def test_terraform_plans_vs_oracle():
    _vs_oracle(synth.tf_corpus(12, start=0, n_resources=40), _pack("tf_rulepack"), "plan")


def test_terraform_full_size_plans_vs_oracle():
    _vs_oracle(synth.tf_corpus(2, start=100, n_resources=2000), _pack("tf_rulepack"), "bigplan")


def test_terraform_full_size_lane_matches_wave():
    docs = synth.tf_corpus(70, start=200, n_resources=600)   # two lane batches, the second ragged
    rules = _pack("tf_rulepack")
    assert _session_report(docs, rules, 0, "p") == _session_report(docs, rules, 1, "p")


def test_config_snapshots_vs_oracle():
    _vs_oracle(synth.config_corpus(24, start=0, n_groups=4), _pack("net_rulepack"), "snapshot")


def test_config_snapshots_lane_matches_wave():
    docs = synth.config_corpus(130, start=1000, n_groups=8)
    rules = _pack("net_rulepack")
    assert _session_report(docs, rules, 0, "s") == _session_report(docs, rules, 1, "s")


def test_container_equality_vs_oracle():
    _vs_oracle(synth.cfn_corpus(16, start=300, n_resources=20), _pack("edge_rulepack"), "doc")


def test_case_converter_queries_vs_oracle():
    # lower-case / snake-case queries over PascalCase templates resolve through the cruet
    # converters (eval_context.rs:539-568); the first document is the one of the reference's
    # test_with_converter (eval_context_tests.rs:407-452)
    from test_oracle_cruet import DOC
    _vs_oracle([DOC] + synth.cfn_corpus(6, start=500, n_resources=12), _pack("conv_rulepack"), "conv")


def test_operator_coverage_vs_oracle():
    # ranges, string ordering, regex ==/!=, !in with a custom message, `some` lets, list and map
    # equality, a named-rule `when` with `not` (tests/golden/ops_rulepack)
    _vs_oracle(synth.cfn_corpus(8, start=700, n_resources=15), _pack("ops_rulepack"), "ops")


def test_cfg1_examples_cross_product_vs_oracle():
    """BASELINE.json configs[0] (the CPU-runnable plumbing case): every guard-examples rules file the
    reference's own test specs use x every template of guard/resources/validate/data-dir, each
    (rules file, template) pair through `validate --structured` on the MI355X and on the oracle"""
    import json
    cases = json.load(open(os.path.join(G, "expectations.json")))
    rules = sorted({(c["rules_name"], c["rules_text"]) for c in cases})
    d = os.path.join(G, "validate", "data-dir")
    data = [(f, open(os.path.join(d, f)).read()) for f in sorted(os.listdir(d))]
    for name, text in rules:
        for dn, dt in data:
            exp, ecode, err = oracle_validate([(name, text)], [(dn, dt)])
            try:
                out, code = guard_amd.validate_structured([(name, text)], [(dn, dt)])
            except guard_amd.GuardError as e:
                assert ecode == -1 and err.endswith("Error occurred " + e.message), (name, dn, e.message)
                continue
            assert (out, code) == (exp, ecode), (name, dn)


def test_sharded_sessions_merge_to_single_process_report():
    """each rank reports its own documents; rank-order concatenation of the
    per-shard reports (sharding.merge_reports, what gather_report does on rank 0) is the
    single-process output.  Two sessions on one GPU stand in for two ranks."""
    import sharding
    from rulepack import rule_pack
    rules = rule_pack()
    texts = synth.cfn_corpus(24, start=100, n_resources=12)
    names = ["synthetic-%d.json" % (100 + i) for i in range(len(texts))]
    for fmt in ("json", "yaml"):
        parts, codes = [], []
        for lo, hi in ((0, 9), (9, 24)):
            s = guard_amd.Session()
            for name, text in rules:
                s.add_rules(text, name)
            s.add_docs(texts[lo:hi], names[lo:hi])
            s.upload()
            s.eval(1)
            out, code = s.report(fmt)
            s.close()
            parts.append(out)
            codes.append(code)
        merged = sharding.merge_reports(parts, fmt)
        exp, ecode, _ = oracle_validate(rules, list(zip(names, texts)), output=fmt)
        assert merged == exp
        assert max(codes, key=lambda c: sharding._SEVERITY[c]) == ecode


def test_key_captures_and_join_reasons_vs_oracle():
    """variable / key captures (`Resources[ id ]`, `Resources[ id | filter ]`) accumulate into the
    root scope and feed joins; join reasons R4 (index past the key list) and R5 (unresolved keys)
    render with their Debug key lists -- byte-identical with the oracle in every format"""
    docs = synth.cfn_corpus(12, start=11, n_resources=6) + synth.cfn_corpus(4, start=90, n_resources=30)
    data = [("cap-%d.json" % i, d) for i, d in enumerate(docs)]
    rules = _pack("capture_rulepack")
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt


def test_key_captures_lane_matches_wave():
    docs = synth.cfn_corpus(130, start=2000, n_resources=20)
    rules = _pack("capture_rulepack")
    assert _session_report(docs, rules, 0, "c") == _session_report(docs, rules, 1, "c")


def test_cfg3_registry_standin_vs_oracle():
    """cfg 3: the full-registry stand-in -- every in-scope in-repo .guard file of the
    reference (tests/golden/cfg3_rulepack, 22 files) -- over synthetic templates, every format"""
    docs = synth.cfn_corpus(24, start=4242, n_resources=50)
    data = [("t-%d.json" % i, d) for i, d in enumerate(docs)]
    rules = _pack("cfg3_rulepack")
    assert len(rules) == 22
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt


def test_cfg3_lane_matches_wave():
    docs = synth.cfn_corpus(130, start=9000, n_resources=50)
    rules = _pack("cfg3_rulepack")
    assert _session_report(docs, rules, 0, "t") == _session_report(docs, rules, 1, "t")


def test_shape_sorted_batch_matches_load_order():
    """Shape-sorted lane batches (capi.cpp session_upload) change only which documents share a
    wavefront: a 640-document cfg-2 batch reports byte-identically with the sort on and off, in every
    format, and equals the oracle on its first documents."""
    import rulepack
    docs = synth.cfn_corpus(640, start=9000, n_resources=50)
    rules = rulepack.rule_pack("cfg2")
    outs = {}
    try:
        for flag in ("1", "0"):
            os.environ["GG_SHAPE_SORT"] = flag
            s = guard_amd.Session()
            for name, text in rules:
                s.add_rules(text, name)
            s.add_docs(docs, ["s-%d.json" % i for i in range(len(docs))])
            s.eval(1)
            outs[flag] = [s.report(fmt) for fmt in ("json", "yaml", "sarif", "junit")]
            s.close()
    finally:
        os.environ.pop("GG_SHAPE_SORT", None)
    assert outs["1"] == outs["0"]
    data = [("s-%d.json" % i, d) for i, d in enumerate(docs[:40])]
    exp, ecode, _ = oracle_validate(rules, data)
    out, code = guard_amd.validate_structured(rules, data)
    assert (code, out) == (ecode, exp)
