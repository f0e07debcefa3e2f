"""The structured JSON report rendered on the MI355X (csrc/report_gpu.hip) against the host writer
(reporter.cpp) and the oracle: the same bytes, document for document, on corpora that exercise every
record kind the device writer covers (rules, disjunctions, unary / binary / IN / block / dependent-rule
clauses, unresolved reasons, literal values, nested values) and the ones it leaves to the host writer
(floats, Debug-formatted reasons, map keys and count() values as values) -- those documents are written by
the host at their positions, so the report never depends on which writer took a document."""
import json
import os

import pytest

import guard_amd
import synth
from guard_oracle import validate_structured as oracle_validate
from rulepack import rule_pack

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _pack_dir(name):
    p = os.path.join(G, name)
    return [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]


def _both(rules, docs, prefix):
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs(docs, ["%s-%d.json" % (prefix, i) for i in range(len(docs))])
    s.eval(1)
    if s.stat(s.STAT["errors"]):
        # an evaluation error aborts both writers alike
        s.set_device_report(True)
        with pytest.raises(guard_amd.GuardError) as a:
            s.report("json")
        s.set_device_report(False)
        with pytest.raises(guard_amd.GuardError) as b:
            s.report("json")
        s.close()
        assert (a.value.code, a.value.message) == (b.value.code, b.value.message)
        return None, None
    s.set_device_report(True)
    dev = s.report("json")
    s.set_device_report(False)
    host = s.report("json")
    n, code, st = s.report_json_device()
    s.close()
    assert dev == host
    assert n == len(host[0].encode()) and code == host[1]
    return dev, st


@pytest.mark.parametrize("pack,corpus", [
    ("cfg2", lambda: synth.cfn_corpus(400, start=77, n_resources=30)),
    ("cfg3", lambda: synth.cfn_corpus(150, start=5000, n_resources=20)),
    ("cfg4", lambda: synth.tf_corpus(10, start=9, n_resources=60)),
    ("cfg5", lambda: synth.config_corpus(120, start=40)),
])
def test_device_report_equals_host_and_oracle(pack, corpus):
    rules = rule_pack(pack)
    docs = corpus()
    (out, code), st = _both(rules, docs, pack)
    assert st["device_docs"] > 0
    data = [("%s-%d.json" % (pack, i), d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    assert (out, code) == (exp, ecode)


@pytest.mark.parametrize("pack", ["capture_rulepack", "edge_rulepack", "ops_rulepack", "count_rulepack", "conv_rulepack",
                                  "unicode_rulepack", "wordb_rulepack", "dupkey_rulepack"])
def test_device_report_packs_equal_host(pack):
    rules = _pack_dir(pack)
    docs = synth.cfn_corpus(60, start=1234, n_resources=12)
    _both(rules, docs, pack)


def test_floats_and_debug_reasons_fall_back_to_host_in_place():
    rules = [("f.guard", "rule r { Resources.*.Properties.Size == 10 }\nrule i { Resources.*.Properties.Items[5] exists }\n"
                         "rule k { Resources.*.Properties.Meta.Foo exists }")]
    docs = []
    for i in range(60):
        size = 2.5 if i % 7 == 0 else (i if i % 5 else "s")         # floats: the host writer
        items = [1, 2] if i % 3 == 0 else [1, 2, 3, 4, 5, 6]        # index out of bounds: Debug of the array
        meta = 5 if i % 4 == 0 else {"Foo": 1}                      # key on a non-struct: Debug of the value
        docs.append(json.dumps({"Resources": {"a": {"Properties": {"Size": size, "Items": items, "Meta": meta}}}}))
    (out, code), st = _both(rules, docs, "f")
    assert st["host_docs"] > 0 and st["device_docs"] > 0
    exp, ecode, _ = oracle_validate(rules, [("f-%d.json" % i, d) for i, d in enumerate(docs)])
    assert (out, code) == (exp, ecode)


def _device_loaded(rules, docs, prefix):
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    st = s.add_docs_device(docs, ["%s-%d.json" % (prefix, i) for i in range(len(docs))])
    assert st is not None, "device loader refused the corpus"
    s.eval(1)
    return s


@pytest.mark.parametrize("resident", ["1", "0"])
def test_resident_arena_reports_equal_oracle(resident, monkeypatch):
    """the device loader leaves the arena's columns in HBM (capi.cpp ensure_host_arena): the device JSON
    report never brings them down; a host writer (YAML, SARIF, a host-fallback document) does, at first
    use -- every format equals the oracle either way"""
    monkeypatch.setenv("GG_RESIDENT_ARENA", resident)
    rules = rule_pack("cfg2")
    docs = synth.cfn_corpus(300, start=4321, n_resources=25)
    data = [("r-%d.json" % i, d) for i, d in enumerate(docs)]
    s = _device_loaded(rules, docs, "r")
    nodes = s.stat(s.STAT["nodes"]) if "nodes" in s.STAT else None
    s.set_device_report(True)
    exp, ecode, _ = oracle_validate(rules, data)
    assert s.report("json") == (exp, ecode)
    for fmt in ("yaml", "sarif"):
        e, c, _ = oracle_validate(rules, data, output=fmt)
        assert s.report(fmt) == (e, c), fmt
    assert s.report("json") == (exp, ecode)
    if nodes is not None:
        assert s.stat(s.STAT["nodes"]) == nodes
    s.close()


def test_resident_arena_host_fallback_documents(monkeypatch):
    monkeypatch.setenv("GG_RESIDENT_ARENA", "1")
    rules = [("f.guard", "rule r { Resources.*.Properties.Size == 10 }\nrule i { Resources.*.Properties.Items[5] exists }")]
    docs = []
    for i in range(80):
        size = 2.5 if i % 7 == 0 else i
        items = [1, 2] if i % 3 == 0 else [1, 2, 3, 4, 5, 6]
        docs.append(json.dumps({"Resources": {"a": {"Properties": {"Size": size, "Items": items}}}}))
    s = _device_loaded(rules, docs, "f")
    s.set_device_report(True)
    n, code, st = s.report_json_device()
    assert st["host_docs"] > 0 and st["device_docs"] > 0
    exp, ecode, _ = oracle_validate(rules, [("f-%d.json" % i, d) for i, d in enumerate(docs)])
    assert s.report("json") == (exp, ecode)
    assert n == len(exp.encode()) and code == ecode
    s.close()


# ------------------------------------------------------------------------------ SARIF on the device ---
def _sarif_both(rules, docs, prefix):
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs(docs, ["%s-%d.json" % (prefix, i) for i in range(len(docs))])
    s.eval(1)
    s.set_device_report(True)
    dev = s.report("sarif")
    s.set_device_report(False)
    host = s.report("sarif")
    # the counted entry the bench's e2e SARIF leg times: the same byte count and exit code
    n, code, st = s.report_sarif_device()
    s.close()
    assert dev == host
    assert n == len(host[0].encode()) and code == host[1]
    return dev


@pytest.mark.parametrize("pack,corpus", [
    ("cfg2", lambda: synth.cfn_corpus(300, start=177, n_resources=30)),
    ("cfg3", lambda: synth.cfn_corpus(120, start=5100, n_resources=20)),
    ("cfg4", lambda: synth.tf_corpus(8, start=19, n_resources=50)),
    ("cfg5", lambda: synth.config_corpus(100, start=60)),
])
def test_device_sarif_equals_host_and_oracle(pack, corpus):
    """SarifReport (sarif.rs:29-53, 127-160, 185-203) with every FAILed document's results rendered on the
    device (report_gpu.hip rg::file_sarif): byte-identical with the host writer and the oracle"""
    rules = rule_pack(pack)
    docs = corpus()
    out, code = _sarif_both(rules, docs, pack)
    data = [("%s-%d.json" % (pack, i), d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data, output="sarif")
    assert (out, code) == (exp, ecode)


@pytest.mark.parametrize("pack", ["capture_rulepack", "edge_rulepack", "ops_rulepack", "count_rulepack", "conv_rulepack",
                                  "unicode_rulepack", "wordb_rulepack", "nfa_rulepack"])
def test_device_sarif_packs_equal_host(pack):
    _sarif_both(_pack_dir(pack), synth.cfn_corpus(60, start=4321, n_resources=12), pack)


def test_device_sarif_host_fallback_documents_and_names():
    """floats / Debug reasons send a document's results to the host writer at its position; repeated and
    empty document names, and names with a leading '/', keep the reference's artifact dedupe and URIs"""
    rules = [("f.guard", "rule r { Resources.*.Properties.Size == 10 }\nrule i { Resources.*.Properties.Items[5] exists }\n"
                         "rule k { Resources.*.Properties.Meta.Foo exists <<custom\nmessage>> }")]
    docs, names = [], []
    for i in range(70):
        size = 2.5 if i % 7 == 0 else (i if i % 5 else "s")
        items = [1, 2] if i % 3 == 0 else [1, 2, 3, 4, 5, 6]
        meta = 5 if i % 4 == 0 else {"Foo": 1}
        docs.append(json.dumps({"Resources": {"a": {"Properties": {"Size": size, "Items": items, "Meta": meta}}}}))
        names.append(["/abs/p%d.json" % (i % 9), "", "rel/q%d.json" % i][i % 3])
    data = list(zip(names, docs))
    exp, ecode, _ = oracle_validate(rules, data, output="sarif")
    out, code = guard_amd.validate_structured(rules, data, output="sarif")
    assert (out, code) == (exp, ecode)
    for devices in ([0, 0], [0, 0, 0]):
        assert guard_amd.validate_structured_devices(rules, data, devices=devices, output="sarif") == (exp, ecode)


def test_device_sarif_golden():
    gdir = os.path.join(G, "validate")
    rules = [(f, open(os.path.join(gdir, "rules-dir", f)).read())
             for f in sorted(os.listdir(os.path.join(gdir, "rules-dir"))) if f.endswith(".guard")]
    dn = "s3-public-read-prohibited-template-non-compliant.yaml"
    out, code = guard_amd.validate_structured(rules, [("some/path", open(os.path.join(gdir, "data-dir", dn)).read())],
                                              output="sarif")
    assert code == 19
    assert out == open(os.path.join(gdir, "structured.sarif")).read()
