"""Block-style YAML on the device loader (csrc/yaml_gpu.inc): the arena it builds equals the host
loader's (libyaml events + scalar typing, doc_loader.cpp; reference Loader::load, libyaml/loader.rs:31-244)
document for document, marks included; documents outside the subset are refused and built by the host at
their positions; reports over device-loaded YAML equal the oracle's."""
import json

import pytest

import guard_amd
import synth
from guard_oracle import validate_structured as oracle_validate
from rulepack import rule_pack

pytestmark = pytest.mark.gpu


def _check(docs):
    rc, msg = guard_amd.loader_device_check(docs)
    assert rc == 1, msg


EDGE = [
    # short-form intrinsics: single-value tags, sequence tags on flow and block sequences, nested flows
    "Resources:\n  B:\n    Type: AWS::S3::Bucket\n    Properties:\n      BucketName: !Ref Name\n"
    "      Arn: !GetAtt B.Arn\n      Joined: !Join [\"-\", [a, b]]\n      Azs: !Select [0, !GetAZs '']\n",
    "x: !Sub 'arn:${AWS::Partition}:s3:::b'\nf: !If\n  - Cond\n  - a\n  - b\nz: !Join\n- ''\n- [a, b]\nw: 1\n",
    "- # a comment after the indicator\n  k: v\n- k2: # and after a key\n    v2\n",
    "u: !Unknown value\nv: !Ref 5\nt: !Ref\n  - a\n",
    # scalar typing: ints (Rust i64::from_str: sign, leading zeros), floats, bools, nulls, strings
    "a:\n- 1\n- two\n- 'three'\n- \"four\"\n- null\n- ~\n- Null\n- true\n- yes\n- off\n- 1.5\n- -7\n- +3\n- 007\n"
    "- 2010-09-09\n- 1e3\n- -0.25E-2\n- 9223372036854775807\n- -9223372036854775808\nb: c\n",
    # empty values, comments, blank lines, trailing spaces
    "k1:\nk2: v\nk3:\n  # c\nk4: x   \n\n\nk5: y # trailing\nk6:\n",
    # compact entries, nested sequences, flow collections, quoted keys
    "list:\n  - a: 1\n    b: 2\n  - - x\n    - y\n  - [1, 2, {z: 3}]\n  - {p: q, 'r': \"s\"}\n\"quoted key\": 'v'\n'k''q': []\nm: {}\n",
    # a leading document marker, comments before it, non-ASCII keys and values
    "# head\n---\n# comment\nroot:\n  k: \"é ü\"\n  ключ: значение\n  e: 😀 ok\n",
    "s: 'it''s'\nt: \"tab\\tand\\u00e9 \\\"q\\\"\"\nu: plain, with commas [and] brackets # c\nv: a:b\n",
    "Resources:\n  X:\n    Type: T\n    DependsOn:\n    - A\n    - B\n    Properties: {}\n    Y: []\n  Z:\n    Type: U\n",
    "- a\n- b: 1\n  c: [x]\n- - 1\n  - 2\n",
    # block scalars: literal / folded, clip / strip / keep, more-indented literal lines, tags, in lists and maps
    "d: |\n  line one\n  line two\n\n  after blank\ne: >\n  folded one\n  folded two\n\n  para\nf: |-\n  strip\n"
    "g: |+\n  keep\n\nh: x\n",
    "u: !Sub |\n  #!/bin/bash\n  echo ${AWS::Region}\n     indented more\n\nv: 1\n",
    "- |\n  in a list\n- >-\n  folded\n  list\n- last\n",
    "k:\n  nested: | # a comment\n    deep\n      deeper\n  next: z\nlast: |\n  at the end",
]


def test_yaml_edge_documents():
    _check(EDGE)
    for d in EDGE:
        _check([d])


def test_yaml_cfn_corpus():
    docs = synth.cfn_yaml_corpus(300, start=11, n_resources=20)
    _check(docs)


def test_mixed_json_and_yaml_batch():
    docs = []
    for i in range(200):
        docs.append(synth.cfn_yaml_doc(500 + i, 8) if i % 3 else json.dumps(synth.cfn_doc(500 + i, 8)))
    _check(docs)


@pytest.mark.parametrize("doc,why", [
    ("a: |2\n  text\n", "YAML subset"),              # an indentation indicator
    ("a: >\n  x\n    more\n", "YAML subset"),          # a more-indented line in a folded scalar
    ("a: |\nb: 1\n", "YAML subset"),                 # an empty block scalar
    ("a: b\n  c\n", "YAML subset"),                   # multi-line plain scalar
    ("a: &x 1\nb: *x\n", "YAML subset"),             # anchors / aliases
    ("a: !!str 1\n", "YAML subset"),                  # a !! tag
    ("a:\n\tb: 1\n", "YAML subset"),                  # tab
    ("a: [1,\n  2]\n", "YAML subset"),               # a flow collection over two lines
    ("a: 1\n---\nb: 2\n", "YAML subset"),             # a second document
    ("a: 1\r\nb: 2\r\n", "YAML subset"),              # CR
    ("? a\n: b\n", "YAML subset"),                    # complex key
    ("a: .5\n", "number"),                            # a float outside the JSON number grammar
    ("a: inf\n", "number"),
    ("a: 99999999999999999999\n", "number"),          # beyond i64: a float to Rust
    ("a: 1\na: 2\n", "duplicate"),
    ("a: 'x\n  y'\n", "YAML subset"),                 # a quoted scalar over two lines
    ("plain scalar document\n", "YAML subset"),
    ("y: 1\n", "YAML subset"),                      # a key the host types (Bool): its error is the host's
    ("1: a\n", "YAML subset"),
    ("a: b#c\nd: x #\ne: 'q'#x\n", "YAML subset"),   # '#' glued to a quoted scalar
])
def test_yaml_refusals(doc, why):
    rc, msg = guard_amd.loader_device_check(synth.cfn_yaml_corpus(2, n_resources=4) + [doc])
    assert rc == -1
    assert why in msg


def test_yaml_off_refuses(monkeypatch):
    monkeypatch.setenv("GG_YAML_DEVICE", "0")
    rc, msg = guard_amd.loader_device_check(synth.cfn_yaml_corpus(2, n_resources=4))
    assert rc == -1 and "JSON" in msg


def test_device_loaded_yaml_reports_equal_oracle():
    rules = rule_pack("cfg2")
    docs = synth.cfn_yaml_corpus(150, start=70, n_resources=20)
    # the oracle types yes / no / on / off as strings: the corpus has none unquoted
    data = [("t-%d.yaml" % i, d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    st = s.add_docs_device(docs, [n for n, _ in data])
    assert st is not None and st["refused_docs"] == 0
    s.eval(1)
    assert s.report("json") == (exp, ecode)
    for fmt in ("yaml", "sarif"):
        e, c, _ = oracle_validate(rules, data, output=fmt)
        assert s.report(fmt) == (e, c), fmt
    s.close()


def test_device_loaded_yaml_with_refused_documents():
    rules = rule_pack("cfg2")
    docs = synth.cfn_yaml_corpus(40, start=900, n_resources=10)
    docs[5] = docs[5].replace("Resources:", "Description: &d anchored\nResources:", 1)   # host-loaded
    docs[17] = docs[17] + "Extra: !Ref Thing\n"
    data = [("r-%d.yaml" % i, d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    st = s.add_docs_device(docs, [n for n, _ in data])
    assert st is not None and st["refused_docs"] == 1
    s.eval(1)
    assert s.report("json") == (exp, ecode)
    s.close()


def test_reference_yaml_fixtures():
    """the reference's own YAML data files (tests/golden, from guard/resources): each one the device takes
    builds the host's arena; the rest are refused, never built differently"""
    import glob
    import os
    root = os.path.join(os.path.dirname(__file__), "golden")
    files = sorted(glob.glob(os.path.join(root, "**", "*.yaml"), recursive=True))
    files = [f for f in files if "rulepack" not in f]
    taken = 0
    for f in files:
        text = open(f, encoding="utf-8").read()
        rc, msg = guard_amd.loader_device_check([text])
        assert rc != 0, (f, msg)
        taken += rc == 1
    assert taken >= 6, taken
    # every template of the reference's validate data-dir loads on the device
    for f in files:
        if os.sep + "data-dir" + os.sep in f:
            assert guard_amd.loader_device_check([open(f, encoding="utf-8").read()])[0] == 1, f
