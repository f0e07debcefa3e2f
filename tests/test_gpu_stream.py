"""cfn_guard_validate_batch_stream (capi.cpp): the structured JSON report streamed through a write callback
while the documents run in chunks on two alternating sessions -- the same bytes and exit code as the
one-string cfn_guard_validate_batch_format call (structured.rs:99-133), whatever the chunk size."""
import json
import os

import pytest

import guard_amd
import synth
from guard_oracle import validate_structured as oracle_validate
from guard_oracle.errors import GuardError, FFI_CODES
from rulepack import rule_pack
from test_gpu_parity import _nfa_docs

G = os.path.join(os.path.dirname(__file__), "golden")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chunk", [1, 7, 64, 100, 0])
def test_stream_equals_one_string(chunk):
    rules = rule_pack("cfg2")
    docs = synth.cfn_corpus(130, start=42, n_resources=12) + synth.cfn_yaml_corpus(40, start=7, n_resources=6)
    data = [("d%d.%s" % (i, "json" if i < 130 else "yaml"), d) for i, d in enumerate(docs)]
    exp = guard_amd.validate_structured(rules, data)
    got = guard_amd.validate_structured_stream(rules, data, chunk_docs=chunk)
    assert got == exp


def test_stream_host_fallback_documents_and_parse_errors():
    rules = rule_pack("cfg2") + [("broken.guard", "rule r { Resources.*.Properties.X == }")]
    docs = synth.cfn_corpus(90, start=3, n_resources=8)
    docs[10] = json.dumps({"Resources": {"a": {"Type": "AWS::S3::Bucket", "Properties": {"Size": 2.5}}}})   # host writer
    docs[70] = "Resources:\n  a: &x\n    Type: AWS::S3::Bucket\n"   # host loader
    data = [("h%d.json" % i, d) for i, d in enumerate(docs)]
    exp = guard_amd.validate_structured(rules, data)
    for chunk in (16, 65, 0):
        assert guard_amd.validate_structured_stream(rules, data, chunk_docs=chunk) == exp


def test_stream_empty_and_error():
    rules = rule_pack("cfg2")
    assert guard_amd.validate_structured_stream(rules, [], chunk_docs=4) == guard_amd.validate_structured(rules, [])
    # a deterministic evaluation error in a later chunk: `empty` on an integer aborts the reference's
    # evaluation (eval.rs:251-262); the streamed entry raises the oracle's code and message
    bad_rules = [("t.guard", "rule r { Resources.*.Properties.Port empty }")]
    docs = synth.cfn_corpus(20, start=1, n_resources=4)
    docs[13] = json.dumps({"Resources": {"b": {"Type": "AWS::S3::Bucket", "Properties": {"Port": 8080}}}})
    data = [("e%d.json" % i, d) for i, d in enumerate(docs)]
    try:
        oracle_validate(bad_rules, data, raise_errors=True)
        raise AssertionError("the oracle did not abort")
    except GuardError as e:
        code, msg = FFI_CODES.get(e.kind, -1), e.display()
    seen = []
    with pytest.raises(guard_amd.GuardError) as g:
        guard_amd.validate_structured_stream(bad_rules, data, write=seen.append, chunk_docs=5)
    assert (g.value.code, g.value.message) == (code, msg)
    with pytest.raises(guard_amd.GuardError) as g1:
        guard_amd.validate_structured(bad_rules, data)
    assert (g1.value.code, g1.value.message) == (code, msg)


def test_stream_vs_oracle():
    """the streamed bytes against the CPU oracle directly (not only against the one-string call, which
    shares the device loader and reporter)"""
    rules = rule_pack("cfg2")
    docs = synth.cfn_corpus(70, start=500, n_resources=9) + synth.cfn_yaml_corpus(30, start=90, n_resources=5)
    data = [("o%d.%s" % (i, "json" if i < 70 else "yaml"), d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    assert guard_amd.validate_structured_stream(rules, data, chunk_docs=24) == (exp, ecode)


def test_nfa_pack_through_stream_and_device_list():
    """regexes past the DFA limits (the NFA kernel variant) through the streamed entry -- two sessions
    alternating, their launches overlapping -- and through a device list [0, 0]: byte-equal to the oracle.
    The variant runs in the default lane stack (no device-wide stack limit is raised for it)."""
    p = os.path.join(G, "nfa_rulepack")
    rules = [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
    data = [("n%d.json" % i, d) for i, d in enumerate(_nfa_docs())]
    exp, ecode, _ = oracle_validate(rules, data)
    for chunk in (9, 40):
        assert guard_amd.validate_structured_stream(rules, data, chunk_docs=chunk) == (exp, ecode), chunk
    assert guard_amd.validate_structured_devices(rules, data, devices=[0, 0], output="json") == (exp, ecode)


def test_stream_callback_failure_aborts():
    rules = rule_pack("cfg2")
    data = [("c%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(30, start=9, n_resources=4))]
    seen = []

    def write(b):
        seen.append(b)
        if len(seen) > 1:
            raise RuntimeError("disk full")
    with pytest.raises(guard_amd.GuardError):
        guard_amd.validate_structured_stream(rules, data, write=write, chunk_docs=10)


def test_synth_texts_inputs_stream():
    rules = rule_pack("cfg2")
    t = guard_amd.SynthTexts(100, 80, n_resources=10, fmt="yaml")
    try:
        got = guard_amd.validate_structured_stream(rules, None, inputs=t.inputs, n_docs=t.n, chunk_docs=30)
    finally:
        t.close()
    data = [("synthetic-%d.yaml" % (100 + i), synth.cfn_yaml_doc(100 + i, 10)) for i in range(80)]
    assert got == guard_amd.validate_structured(rules, data)


def test_device_block_cache_reuse_and_release():
    """dev_cache.h: loader temporaries and session buffers freed to the per-device cache are reused dirty by
    later calls (a different batch in between) with the same bytes as fresh blocks; the release entry
    empties the cache."""
    rules = rule_pack("cfg2")
    a = [("a%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(150, start=5, n_resources=9))]
    b = [("b%d.yaml" % i, d) for i, d in enumerate(synth.cfn_yaml_corpus(120, start=77, n_resources=11))]
    assert guard_amd.release_device_cache() >= 0
    assert guard_amd.release_device_cache() == 0
    exp_a = guard_amd.validate_structured(rules, a)    # fresh blocks
    exp_b = guard_amd.validate_structured(rules, b)    # some of a's blocks, dirty
    assert guard_amd.validate_structured(rules, a) == exp_a
    assert guard_amd.validate_structured_stream(rules, a + b, chunk_docs=64) == guard_amd.validate_structured(rules, a + b)
    assert guard_amd.validate_structured(rules, b) == exp_b
    assert guard_amd.release_device_cache(0) > 0
    assert guard_amd.release_device_cache(-1) == 0


@pytest.mark.parametrize("devices,chunk", [([0, 0], 7), ([0, 0, 0], 32), ([0], 16), (None, 50)])
def test_stream_devices_equals_one_device_and_oracle(devices, chunk):
    """cfn_guard_validate_batch_stream_devices: chunks spread over a device list (ordinals repeat on the
    one-GPU box: separate pipelines, sessions and streams on one device), written in document order -- the
    one-device stream's bytes and the oracle's"""
    rules = rule_pack("cfg2")
    docs = synth.cfn_corpus(110, start=300, n_resources=7) + synth.cfn_yaml_corpus(25, start=40, n_resources=5)
    data = [("m%d.%s" % (i, "json" if i < 110 else "yaml"), d) for i, d in enumerate(docs)]
    exp, ecode, _ = oracle_validate(rules, data)
    assert guard_amd.validate_structured_stream(rules, data, chunk_docs=chunk) == (exp, ecode)
    assert guard_amd.validate_structured_stream(rules, data, chunk_docs=chunk, devices=devices) == (exp, ecode)


def test_stream_devices_errors_and_empty():
    rules = rule_pack("cfg2")
    assert (guard_amd.validate_structured_stream(rules, [], chunk_docs=4, devices=[0, 0])
            == guard_amd.validate_structured(rules, []))
    bad_rules = [("t.guard", "rule r { Resources.*.Properties.Port empty }")]
    docs = synth.cfn_corpus(30, start=2, n_resources=4)
    docs[21] = json.dumps({"Resources": {"b": {"Type": "AWS::S3::Bucket", "Properties": {"Port": 8080}}}})
    data = [("x%d.json" % i, d) for i, d in enumerate(docs)]
    with pytest.raises(guard_amd.GuardError) as g1:
        guard_amd.validate_structured_stream(bad_rules, data, chunk_docs=4)
    with pytest.raises(guard_amd.GuardError) as g2:
        guard_amd.validate_structured_stream(bad_rules, data, chunk_docs=4, devices=[0, 0])
    assert (g1.value.code, g1.value.message) == (g2.value.code, g2.value.message)
    seen = []

    def write(b):
        seen.append(b)
        if len(seen) > 1:
            raise RuntimeError("disk full")
    with pytest.raises(guard_amd.GuardError):
        guard_amd.validate_structured_stream(rule_pack("cfg2"), data, write=write, chunk_docs=5, devices=[0, 0])
    with pytest.raises(guard_amd.GuardError):
        guard_amd.validate_structured_stream(rules, data, chunk_docs=5, devices=[])


# ---- round 6: cfn_guard_validate_batch_stream_ex -- every structured format and -i on the streamed entries
def _mixed_corpus(n_json, n_yaml, start):
    docs = synth.cfn_corpus(n_json, start=start, n_resources=8) + synth.cfn_yaml_corpus(n_yaml, start=start + 3, n_resources=5)
    return [("f%d.%s" % (i, "json" if i < n_json else "yaml"), d) for i, d in enumerate(docs)]


@pytest.mark.parametrize("output", ["yaml", "sarif", "junit", "json"])
@pytest.mark.parametrize("chunk", [1, 9, 0])
def test_stream_every_format_equals_one_string_and_oracle(output, chunk):
    rules = rule_pack("cfg2")
    data = _mixed_corpus(50, 14, 120)
    one = guard_amd.validate_structured(rules, data, output=output)
    params = [("p.yaml", "Extra:\n  Note: x\n")] if output == "json" else None   # json: the -i path of the entry
    if params:
        one = guard_amd.validate_structured(rules, data, output=output, params=params)
    got = guard_amd.validate_structured_stream(rules, data, chunk_docs=chunk, output=output, params=params)
    assert got == one
    exp, ecode, _ = oracle_validate(rules, data, output=output, params=params)
    assert got == (exp, ecode)


@pytest.mark.parametrize("output", ["yaml", "sarif", "junit"])
def test_stream_formats_with_params_and_device_list(output):
    rules = rule_pack("cfg2") + [("p.guard", "rule uses_param { Extra.Note == 'x' }")]
    data = _mixed_corpus(30, 6, 7)
    params = [("p1.yaml", "Extra:\n  Note: x\n"), ("p2.json", '{"Other": 1}')]
    one = guard_amd.validate_structured(rules, data, output=output, params=params)
    assert guard_amd.validate_structured_stream(rules, data, chunk_docs=8, output=output, params=params) == one
    assert guard_amd.validate_structured_stream(rules, data, chunk_docs=5, output=output, params=params, devices=[0, 0]) == one


@pytest.mark.parametrize("output", ["yaml", "sarif", "junit", "json"])
def test_stream_formats_empty_parse_error_and_errors(output):
    rules = rule_pack("cfg2") + [("broken.guard", "rule r { Resources.*.Properties.X == }")]
    assert guard_amd.validate_structured_stream(rules, [], chunk_docs=4, output=output) == \
        guard_amd.validate_structured(rules, [], output=output)
    data = _mixed_corpus(20, 4, 55)
    assert guard_amd.validate_structured_stream(rules, data, chunk_docs=6, output=output) == \
        guard_amd.validate_structured(rules, data, output=output)
    # an evaluation error in a later chunk and a load error after it: the one-string call's error (the load error)
    bad_rules = [("t.guard", "rule r { Resources.*.Properties.Port empty }")]
    docs = [d for _, d in _mixed_corpus(24, 0, 3)]
    docs[9] = json.dumps({"Resources": {"b": {"Type": "AWS::S3::Bucket", "Properties": {"Port": 8080}}}})
    docs[20] = '{"Resources": '   # does not load
    bad = [("e%d.json" % i, d) for i, d in enumerate(docs)]
    with pytest.raises(guard_amd.GuardError) as g1:
        guard_amd.validate_structured(bad_rules, bad, output=output)
    seen = []
    with pytest.raises(guard_amd.GuardError) as g2:
        guard_amd.validate_structured_stream(bad_rules, bad, write=seen.append, chunk_docs=5, output=output)
    assert (g1.value.code, g1.value.message) == (g2.value.code, g2.value.message)
    if output in ("sarif", "junit"):
        assert not seen   # SARIF / JUnit write nothing before an error
    # a parameter file that does not load, with every data file loading: the parameter error
    with pytest.raises(guard_amd.GuardError) as g3:
        guard_amd.validate_structured(rules, data, output=output, params=[("bad.yaml", "a: [")])
    with pytest.raises(guard_amd.GuardError) as g4:
        guard_amd.validate_structured_stream(rules, data, output=output, params=[("bad.yaml", "a: [")], chunk_docs=7)
    assert (g3.value.code, g3.value.message) == (g4.value.code, g4.value.message)
