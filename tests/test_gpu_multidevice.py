"""Multi-GPU behind the C ABI (cfn_guard_validate_batch_devices; SURVEY.md 8(b) n_gpus, 8(e)): the
documents sharded over a device list inside the library -- contiguous byte-balanced ranges, one host
thread + device per shard, reports joined in document order -- must give the one-device call's bytes and
exit code in every format.  On the one-GPU box the device list repeats ordinal 0 (two / three / five
shards on one GPU): the same code path as distinct devices, each shard with its own device buffers,
stream and session.  Error precedence (first unloadable document, parameter errors, first erroring
tile) is checked against the one-device call too."""
import os

import pytest

import guard_amd
import synth
from rulepack import rule_pack

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
FMTS = ("json", "yaml", "sarif", "junit")


def _dir(sub, ext):
    d = os.path.join(G, sub)
    return [(f, open(os.path.join(d, f)).read()) for f in sorted(os.listdir(d)) if f.endswith(ext)]


def _same(rules, data, devices, params=None):
    for fmt in FMTS:
        one = guard_amd.validate_structured(rules, data, output=fmt, params=params)
        many = guard_amd.validate_structured_devices(rules, data, devices=devices, output=fmt, params=params)
        assert many == one, (fmt, devices)


def test_cfg2_corpus_sharded_like_one_device():
    docs = synth.cfn_corpus(300, start=11)
    data = [("synthetic-%d.json" % i, d) for i, d in enumerate(docs)]
    rules = rule_pack("cfg2")
    for devices in ([0, 0], [0, 0, 0], [0] * 5):
        _same(rules, data, devices)


def test_reference_data_dir_sharded_like_one_device():
    rules = [r for r in _dir(os.path.join("validate", "rules-dir"), ".guard") if "lookbehind" not in r[0]]
    data = _dir(os.path.join("validate", "data-dir"), ".yaml")
    _same(rules, data, [0, 0])
    _same(rules, data, [0] * 8)        # more shards than documents: idle shards report nothing


def test_terraform_and_capture_packs_sharded():
    docs = synth.tf_corpus(9, start=3, n_resources=60)
    _same(rule_pack("cfg4"), [("plan-%d.json" % i, d) for i, d in enumerate(docs)], [0, 0, 0])
    cap = _dir("capture_rulepack", ".guard")
    cdocs = synth.cfn_corpus(40, start=900)
    _same(cap, [("c-%d.json" % i, d) for i, d in enumerate(cdocs)], [0, 0])


def test_input_parameters_sharded():
    P = os.path.join(G, "params")
    rules = [("db_param_port_rule.guard", open(os.path.join(P, "db_param_port_rule.guard")).read())]
    data = [("db_resource.yaml", open(os.path.join(P, "db_resource.yaml")).read())] * 3
    params = [(f, open(os.path.join(P, "input-parameters-dir", f)).read()) for f in ("db_params.yaml",)]
    _same(rules, data, [0, 0], params=params)


def _error(fn):
    with pytest.raises(guard_amd.GuardError) as ei:
        fn()
    return ei.value.code, ei.value.message


def test_error_precedence_matches_one_device():
    rules = rule_pack("cfg2")
    good = synth.cfn_corpus(6, start=5)
    bad = "Resources: [unclosed"
    # an unloadable document in the last shard: the same load error as the one-device run
    data = [("d%d.json" % i, d) for i, d in enumerate(good)] + [("bad.yaml", bad)]
    one = _error(lambda: guard_amd.validate_structured(rules, data))
    many = _error(lambda: guard_amd.validate_structured_devices(rules, data, devices=[0, 0, 0]))
    assert many == one
    # an evaluation error (EMPTY on an int) in a later shard: the first erroring tile's error
    erules = [("e.guard", "rule r { Resources.*.Properties.Size EMPTY }")]
    edata = [("a.json", '{"Resources": {"x": {"Properties": {"Size": [1]}}}}'),
             ("b.json", '{"Resources": {"y": {"Properties": {"Size": 3}}}}'),
             ("c.json", '{"Resources": {"z": {"Properties": {"Size": 4}}}}')]
    one = _error(lambda: guard_amd.validate_structured(erules, edata))
    many = _error(lambda: guard_amd.validate_structured_devices(erules, edata, devices=[0, 0, 0]))
    assert many == one


def test_unparsable_rules_file_exit_code_sharded():
    rules = rule_pack("cfg2")[:2] + [("broken.guard", "rule x { Resources.* == }")]
    data = [("d%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(8, start=70))]
    _same(rules, data, [0, 0])


def test_bad_device_list_is_an_error():
    code, msg = _error(lambda: guard_amd.validate_structured_devices(rule_pack("cfg2"), [("a.json", "{}")],
                                                                      devices=[0, 99]))
    assert code == -1 and "out of range" in msg
