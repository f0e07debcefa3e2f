"""The device loader (csrc/json_gpu.hip) against the host loader and the oracle.

* arena parity: gg_loader_device_check builds the same documents with both loaders and compares
  every node (kind, count, links, scalars, marks, string bytes, one pool entry per distinct string);
* raw UTF-8: strings with non-ASCII characters load on the device with libyaml's character-counted
  column marks;
* refusals: a document outside the device subset (a YAML document, duplicate keys, nesting past 64, a
  float beyond the exact fast path, a raw character libyaml reads specially) is refused on its own:
  the session builds it with the host loader at its position (the strict check refuses the batch);
* end to end: a session loaded on the device reports byte-identically to one loaded on the host,
  and to the oracle.
"""
import json
import os

import pytest

import guard_amd
import synth
from guard_oracle import validate_structured as oracle_validate
from rulepack import rule_pack

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _pack(d):
    p = os.path.join(G, d)
    return [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]


EDGE_DOCS = [
    '{}', '[]', '  {\n  "a" : [ ] ,\n "b":{ } }\n', '[1, -2, 0, -0, 9223372036854775807, -9223372036854775808]',
    '{"f": [1.5, -0.0, 0.1, 1e3, 2.5E-3, 123456789012345, 0.000123, 1e22, 1e-22, 100.25]}',
    '{"s": ["", "x", "\\u00e9t\\u00e9", "\\u4e2d", "a\\"b\\\\c\\/d\\b\\f\\n\\r\\t", "\\u0041"], "": "", "e": ""}',
    '{"Resources": {"r": {"Type": "T", "Properties": {"": 1, "Name": 2}}}}',
    '[[[[[[[[[[{"deep": [true, false, null]}]]]]]]]]]]',
    '{"k1": {"k1": {"k1": "k1"}}, "k2": ["k1", "k2", {"k2": "k1"}]}',
]


def _check(docs):
    rc, msg = guard_amd.loader_device_check(docs)
    assert rc == 1, msg


def test_arena_parity_edge_documents():
    _check(EDGE_DOCS)
    for d in EDGE_DOCS:
        _check([d])


def test_arena_parity_corpora():
    _check(synth.cfn_corpus(64, start=0, n_resources=30))
    _check(synth.tf_corpus(8, start=5, n_resources=120))
    _check(synth.config_corpus(16, start=3, n_groups=4))


def test_arena_parity_wide_maps():
    """maps of 50-250 distinct keys (the duplicate-key filter sees colliding bits) and a 65535-element list"""
    docs = ["{" + ", ".join('"key-%d-%d": %d' % (n, i, i) for i in range(n)) + "}" for n in (50, 130, 250)]
    docs.append("[" + ",".join(["0"] * 65535) + "]")
    _check(docs)


def test_arena_parity_exact_floats():
    """floats beyond Clinger's fast path (more than 15 digits, large exponents, subnormals) parse on the
    device by Eisel-Lemire, bit-identical to the host loader's"""
    _check(['{"f": [0.12345678901234567890, 2.2250738585072014e-308, 4.9e-324, 123456789012345678.5, '
            '1.7976931348623157e308, 0.30000000000000004, 9007199254740993.0, 1e-400, 3.141592653589793238462643]}',
            '[1.0000000000000002, 0.1e-5, 5e-324, 2.4703282292062328e-324, 6.02214076e23]'])


def test_arena_parity_pretty_printed():
    """multi-line documents: line / column marks of keys and values"""
    docs = [json.dumps(json.loads(d), indent=k) for k, d in
            zip([1, 2, 4, 2, 3, 2], synth.cfn_corpus(6, start=40, n_resources=10))]
    docs += [json.dumps(json.loads(d), indent=2) for d in synth.tf_corpus(2, start=9, n_resources=20)]
    _check(docs)


def test_arena_parity_fixture_json():
    """the JSON fixtures the reference's tests hold (a test spec, structured reports): pretty-printed"""
    paths = [os.path.join(G, "test-command", "s3_bucket_server_side_encryption_enabled.json"),
             os.path.join(G, "validate", "structured.json"), os.path.join(G, "validate", "structured-payload.json")]
    docs = [open(p).read() for p in paths]
    good = [t for t in docs if guard_amd.loader_device_check([t])[0] == 1]
    assert len(good) >= 2
    _check(good)


@pytest.mark.parametrize("doc,why", [
    ("Resources: &x\n  a: 1\n", "YAML subset"),   # an anchor: outside the YAML subset too
    ('{"a": 1, "a": 2}', "duplicate"),
    ("[" * 70 + "]" * 70, "deeper"),
    ('{"x": 1e400}', "float"),
    ('{"x": 99999999999999999999}', "float"),
    ('{"x": 1}x', "subset"),
    ('{"x": "a\u0085b"}', "subset"),   # raw NEL: a line break to libyaml
    ('{"x": "a\u2028b"}', "subset"),   # raw LINE SEPARATOR
    ('{"x": "a\u0090b"}', "subset"),   # raw C1 control: libyaml rejects it
    ("{" + ", ".join('"k%d": %d' % (i, i) for i in range(100)) + ', "k37": 0}', "duplicate"),   # past the key filter
    ("[" + ",".join(["1"] * 70000) + "]", "65535"),   # child counts are 16-bit on the device
])
def test_refusals(doc, why):
    rc, msg = guard_amd.loader_device_check(synth.cfn_corpus(3, n_resources=5) + [doc])
    assert rc == -1
    assert why in msg


UTF8_DOCS = [
    '{"x": "café", "ключ": "значение", "e": "😀 ok", "t": "中文字符", "n": "\u00a0nbsp"}',
    '{"Resources": {"Bücket": {"Type": "AWS::S3::Bucket", "Properties": {"Tags": [{"Key": "ñame", "Value": "日本"}], '
    '"BucketName": "x"}}}}',
]


def test_arena_parity_utf8():
    """raw UTF-8 strings on the device; pretty-printed, so keys and values after a non-ASCII character
    on the same line check the character-counted columns"""
    docs = UTF8_DOCS + [json.dumps(json.loads(d), indent=2, ensure_ascii=False) for d in UTF8_DOCS]
    docs += [json.dumps({"a": "é" * 40, "b": ["ü", {"c": "😀😀", "d": 1}]}, ensure_ascii=False)]
    _check(docs)
    for d in docs:
        _check([d])


def test_session_refused_documents_load_on_the_host():
    """documents the device refuses are built by the host loader at their positions: the session's
    report equals a host-loaded session's and the oracle's"""
    rules = rule_pack()
    base = synth.cfn_corpus(12, start=700, n_resources=15)
    odd = ['Resources:\n  b:\n    Type: AWS::S3::Bucket\n    Properties: {BucketName: x}\n    Metadata: &a x\n',
           '{"Resources": {"a": {"Type": "AWS::S3::Bucket"}, "a": {"Type": "AWS::IAM::Role"}}}',
           '{"Resources": {"v": {"Type": "AWS::EC2::Volume", "Properties": {"Size": 99999999999999999999}}}}',
           UTF8_DOCS[1]]
    texts = base[:3] + [odd[0]] + base[3:7] + odd[1:3] + base[7:] + [odd[3]]
    names = ["m%d.json" % i for i in range(len(texts))]
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    st = s.add_docs_device(texts, names)
    assert st is not None and st["refused_docs"] == 3   # the anchored YAML, duplicate-key and beyond-u64 documents
    s.eval(1)
    dev = s.report()
    s.close()
    assert dev == _session(rules, texts, names, False)
    exp, ecode, _ = oracle_validate(rules, list(zip(names, texts)))
    assert dev == (exp, ecode)


def test_device_then_host_documents_in_one_session():
    """the device loader's nodes stay in HBM for the upload; documents the host loader appends after
    them (and refused ones) cross PCIe on their own: the report equals an all-host session's"""
    rules = rule_pack()
    dev_texts = synth.cfn_corpus(10, start=900, n_resources=12) + [
        '{"Resources": {"a": {"Type": "AWS::S3::Bucket"}, "a": {"Type": "AWS::IAM::Role"}}}']
    host_texts = synth.cfn_corpus(5, start=950, n_resources=9)
    names = ["d%d.json" % i for i in range(len(dev_texts) + len(host_texts))]
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    st = s.add_docs_device(dev_texts, names[:len(dev_texts)])
    assert st is not None and st["refused_docs"] == 1
    s.add_docs(host_texts, names[len(dev_texts):])
    s.eval(1)
    got = s.report()
    s.close()
    assert got == _session(rules, dev_texts + host_texts, names, False)


def _session(rules, texts, names, device):
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    if device:
        st = s.add_docs_device(texts, names)
        assert st is not None and st["text_bytes"] == sum(len(t) for t in texts)
    else:
        s.add_docs(texts, names)
    s.eval(1)
    out = s.report()
    s.close()
    return out


def test_session_device_load_matches_host_and_oracle():
    rules = rule_pack()
    texts = synth.cfn_corpus(40, start=500, n_resources=25)
    names = ["t%d.json" % i for i in range(len(texts))]
    dev = _session(rules, texts, names, True)
    assert dev == _session(rules, texts, names, False)
    exp, ecode, _ = oracle_validate(rules, list(zip(names, texts)))
    assert dev == (exp, ecode)


def test_session_device_load_workloads():
    for texts, rules in ((synth.tf_corpus(6, start=11, n_resources=60), _pack("tf_rulepack")),
                         (synth.config_corpus(10, start=21), _pack("net_rulepack")),
                         (EDGE_DOCS[2:], _pack("edge_rulepack"))):
        names = ["d%d.json" % i for i in range(len(texts))]
        dev = _session(rules, texts, names, True)
        assert dev == _session(rules, texts, names, False)


def test_empty_key_does_not_alias_next_string():
    """an empty string takes its own pool slot (before: "" and the next interned string shared an id)"""
    rules = [("empty.guard", "rule names_two { Resources.*.Properties.Name == 2 }\n")]
    data = [("e.json", EDGE_DOCS[6])]
    exp, ecode, _ = oracle_validate(rules, data)
    assert guard_amd.validate_structured(rules, data) == (exp, ecode)
    assert _session(rules, [EDGE_DOCS[6]], ["e.json"], True) == (exp, ecode)


def test_synthetic_device_matches_host():
    rules = rule_pack()
    a = guard_amd.Session()
    b = guard_amd.Session()
    for name, text in rules:
        a.add_rules(text, name)
        b.add_rules(text, name)
    st = a.add_synthetic_device(1000, 300, n_resources=50)
    assert st is not None and st["nodes"] == a.stat(2)
    b.add_synthetic(1000, 300, n_resources=50)
    assert a.stat(2) == b.stat(2)
    a.eval(1)
    b.eval(1)
    assert a.report() == b.report()
    a.close()
    b.close()


def test_fingerprint_collisions_are_caught(monkeypatch):
    """fingerprints narrowed to 4 bits (GG_JSON_FP_MASK): different strings share table slots, the
    verification finds every occurrence whose bytes differ from its slot's pool string, and the
    document is refused -- the strict check names the collision, a session loads those documents on
    the host and reports as a host-loaded session does"""
    monkeypatch.setenv("GG_JSON_FP_MASK", "0xF")
    # lists of strings: no map, so no duplicate-key check sees the shared slots first
    rc, msg = guard_amd.loader_device_check(['["alpha-%d", "beta-%d", "gamma-%d"]' % (i, i, i) for i in range(10)])
    assert rc == -1 and "collision" in msg
    # templates: keys of one map that share a slot read as duplicates first; either way refused
    docs = synth.cfn_corpus(6, start=11, n_resources=8)
    rules = rule_pack()
    names = ["c%d.json" % i for i in range(len(docs))]
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    st = s.add_docs_device(docs, names)
    assert st is not None and st["refused_docs"] >= 1
    s.eval(1)
    dev = s.report()
    s.close()
    monkeypatch.delenv("GG_JSON_FP_MASK")
    assert dev == _session(rules, docs, names, False)


def test_intern_table_doubles_when_full(monkeypatch):
    """The device intern table starts small (cache-resident probes) and doubles when a batch has
    more distinct strings than it holds; the arena is still the host loader's."""
    monkeypatch.setenv("GG_JSON_TABLE_LOG", "16")
    docs = ['{"k%d": ["%s"]}' % (i, '", "'.join("v%d-%d" % (i, j) for j in range(60))) for i in range(1500)]
    _check(docs)
    s = guard_amd.Session()
    st = s.add_docs_device(docs, ["d%d.json" % i for i in range(len(docs))])
    s.close()
    assert st is not None and st["table_retries"] >= 1 and st["distinct_strings"] == 1500 * 61


def test_key_fingerprint_collision_is_a_collision(monkeypatch):
    """two different keys of one map sharing a narrowed fingerprint: the verify pass names the collision
    (BAD_VERIFY), not a duplicate key; a true duplicate stays a duplicate"""
    monkeypatch.setenv("GG_JSON_FP_MASK", "0x1")
    doc = "{" + ", ".join('"key-%d": %d' % (i, i) for i in range(12)) + "}"
    rc, msg = guard_amd.loader_device_check([doc])
    assert rc == -1 and "collision" in msg, msg
    monkeypatch.delenv("GG_JSON_FP_MASK")
    rc, msg = guard_amd.loader_device_check(['{"a": 1, "b": 2, "a": 3}'])
    assert rc == -1 and "duplicate" in msg, msg


def test_wide_map_reason():
    doc = "{" + ", ".join('"k%d": %d' % (i, i) for i in range(300)) + "}"
    rc, msg = guard_amd.loader_device_check([doc])
    assert rc == -1 and "more than 256 keys" in msg, msg
