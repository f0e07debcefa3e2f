"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle and the reference goldens.

Bit-exact on bytes: every comparison is on the full structured JSON text.
"""
import json
import os

import pytest

import guard_amd
import synth
from guard_oracle import validate_structured as oracle_validate
from guard_oracle import run_checks as oracle_run_checks
from rulepack import rule_pack

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _rules_dir():
    d = os.path.join(G, "validate", "rules-dir")
    return [(f, open(os.path.join(d, f)).read()) for f in sorted(os.listdir(d)) if f.endswith(".guard")]


def test_structured_json_golden():
    dn = "s3-public-read-prohibited-template-non-compliant.yaml"
    data = [(dn, open(os.path.join(G, "validate", "data-dir", dn)).read())]
    out, code = guard_amd.validate_structured(_rules_dir(), data)
    assert code == 19
    assert out == open(os.path.join(G, "validate", "structured.json")).read()


def _data_dir():
    d = os.path.join(G, "validate", "data-dir")
    return [(f, open(os.path.join(d, f)).read()) for f in sorted(os.listdir(d)) if f.endswith(".yaml")]


def test_all_data_dir_vs_oracle():
    """validate/rules-dir x validate/data-dir.  The three rules files without look-around x all six
    templates: byte-identical in every format.  The look-behind rules file alone x each template:
    byte-identical where the oracle never evaluates the look-behind regex, and the explicit
    "unsupported on MI355X path" error exactly where it does."""
    from guard_oracle import rxcompat
    rules = _rules_dir()
    plain = [r for r in rules if "lookbehind" not in r[0]]
    fancy = [r for r in rules if "lookbehind" in r[0]]
    assert len(plain) == 3 and len(fancy) == 1
    data = _data_dir()
    assert len(data) == 6
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(plain, data, output=fmt)
        out, code = guard_amd.validate_structured(plain, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt
    reached = 0
    for dn, text in data:
        rxcompat.EVALUATED.clear()
        exp, ecode, _ = oracle_validate(fancy, [(dn, text)])
        if any(rxcompat.fancy_only(p) for p in rxcompat.EVALUATED):
            reached += 1
            with pytest.raises(guard_amd.GuardError) as ei:
                guard_amd.validate_structured(fancy, [(dn, text)])
            assert ei.value.code == -1 and "unsupported on MI355X path" in ei.value.message
            continue
        out, code = guard_amd.validate_structured(fancy, [(dn, text)])
        assert (code, out) == (ecode, exp), dn
    assert reached == 2   # the two advanced_regex_negative_lookbehind_* templates


def test_structured_payload_golden():
    from test_oracle_golden import COMPLIANT_PAYLOAD_DATA
    rules = [("RULES_STDIN[1]", 'Parameters.InstanceName == "TestInstance"'),
             ("RULES_STDIN[2]", 'Parameters.InstanceName == "TestInstance"')]
    data = [("DATA_STDIN[1]", COMPLIANT_PAYLOAD_DATA), ("DATA_STDIN[2]", COMPLIANT_PAYLOAD_DATA)]
    out, code = guard_amd.validate_structured(rules, data)
    assert code == 0
    assert out == open(os.path.join(G, "validate", "structured-payload.json")).read()


def test_reference_test_specs_vs_oracle():
    cases = json.load(open(os.path.join(G, "expectations.json")))
    bad = []
    for c in cases:
        rules = [(c["rules_name"], c["rules_text"])]
        data = [("input-%d.json" % c["case"], c["input_json"])]
        exp, ecode, eerr = oracle_validate(rules, data)
        try:
            out, code = guard_amd.validate_structured(rules, data)
        except guard_amd.GuardError as e:
            out, code = "ERR " + e.message, -1
        if out != exp or code != ecode:
            bad.append((c["spec"], c["case"], code, ecode))
    assert not bad, bad[:10]


def test_run_checks_ffi_vs_oracle():
    docs = synth.cfn_corpus(4, start=1000, n_resources=12)
    for name, text in rule_pack():
        for i, d in enumerate(docs):
            exp = oracle_run_checks(d, "doc%d.json" % i, text, name)
            got = guard_amd.run_checks(d, "doc%d.json" % i, text, name)
            assert got == exp, (name, i)


def test_synthetic_corpus_vs_oracle():
    docs = synth.cfn_corpus(24, start=0, n_resources=20)
    data = [("doc%d.json" % i, d) for i, d in enumerate(docs)]
    rules = rule_pack()
    exp, ecode, _ = oracle_validate(rules, data)
    out, code = guard_amd.validate_structured(rules, data)
    assert code == ecode
    assert out == exp


def test_session_large_batch_statuses_vs_oracle():
    """Batch of 256 docs through the session API; per-tile statuses vs the oracle."""
    from guard_oracle.parser import parse_rules
    from guard_oracle.loader import load_document
    from guard_oracle import evaluator as E
    docs = synth.cfn_corpus(256, start=5000, n_resources=50)
    rules = rule_pack()
    s = guard_amd.Session()
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs(docs, ["d%d" % i for i in range(len(docs))])
    s.eval(1)
    assert s.stat(s.STAT["errors"]) == 0
    st = s.tile_status(len(docs) * len(rules))
    parsed = [parse_rules(t, n) for n, t in rules]
    want = {"PASS": 0, "FAIL": 1, "SKIP": 2}
    for i, d in enumerate(docs[:64]):
        doc = load_document(d, "d%d" % i)
        for f, rf in enumerate(parsed):
            root = E.RootScope(rf, doc)
            status = E.eval_rules_file(rf, root, "d%d" % i)
            assert st[i * len(rules) + f] == want[status], (i, f)


def _session_report(docs, rules, mode, lane_heap=0):
    s = guard_amd.Session()
    s.configure(mode, lane_heap)
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs(docs, ["synthetic-%d.json" % i for i in range(len(docs))])
    s.eval(1)
    out, code = s.report()
    retried = s.stat(s.STAT["retried"])
    s.close()
    return out, code, retried


@pytest.mark.gpu
def test_lane_mode_matches_wave_mode():
    """One-tile-per-lane and one-tile-per-wavefront kernels produce byte-identical reports."""
    docs = synth.cfn_corpus(130, start=777, n_resources=50)   # 3 lane batches, last one ragged
    rules = rule_pack()
    lane, lcode, _ = _session_report(docs, rules, 0)
    wave, wcode, _ = _session_report(docs, rules, 1)
    assert lcode == wcode
    assert lane == wave


@pytest.mark.gpu
def test_lane_overflow_retried_in_wave_mode():
    """Tiles that outgrow the lane heap are re-run in wave mode; results unchanged."""
    docs = synth.cfn_corpus(8, start=31, n_resources=200)
    rules = rule_pack()
    lane, lcode, retried = _session_report(docs, rules, 0, 32 * 1024)
    wave, wcode, _ = _session_report(docs, rules, 1)
    assert retried > 0
    assert (lane, lcode) == (wave, wcode)


@pytest.mark.gpu
def test_structured_yaml_sarif_junit_goldens():
    """-o yaml / sarif / junit (guard/tests/validate.rs:597-631) through the C ABI"""
    import re
    dn = "s3-public-read-prohibited-template-non-compliant.yaml"
    data = [(dn, open(os.path.join(G, "validate", "data-dir", dn)).read())]
    for fmt in ("json", "yaml", "sarif", "junit"):
        out, code = guard_amd.validate_structured(_rules_dir(), data, output=fmt)
        assert code == 19
        if fmt == "sarif":
            out = re.sub(r'("uri": ".*")', '"uri": "some/path"', out)   # tests/utils.rs:82-90
        assert out == open(os.path.join(G, "validate", "structured." + fmt)).read(), fmt


@pytest.mark.gpu
def test_output_formats_vs_oracle():
    """every output format over the synthetic corpus and the cfg-4 / cfg-5 packs, against the oracle"""
    def pack(d):
        p = os.path.join(G, d)
        return [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
    cases = [
        ([("doc%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(8, start=40, n_resources=15))], rule_pack()),
        ([("/plans/p%d.json" % i, d) for i, d in enumerate(synth.tf_corpus(4, start=7, n_resources=20))], pack("tf_rulepack")),
        ([("snap%d.json" % i, d) for i, d in enumerate(synth.config_corpus(4, start=9))], pack("net_rulepack")),
        ([("doc%d.json" % i, d) for i, d in enumerate(synth.cfn_corpus(4, start=300, n_resources=20))], pack("edge_rulepack")),
    ]
    for data, rules in cases:
        for fmt in ("yaml", "sarif", "junit"):
            exp, ecode, _ = oracle_validate(rules, data, output=fmt)
            out, code = guard_amd.validate_structured(rules, data, output=fmt)
            assert (out, code) == (exp, ecode), (fmt, rules[0][0])


def test_device_selection_env_out_of_range_fails_loudly():
    """One device per process: GG_DEVICE (or the caller's current device) picks it; an ordinal past
    the visible devices is an error (-1), never a silent fallback to another device or the CPU."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import guard_amd\n"
            "try:\n    guard_amd.validate_structured([('r.guard', 'Resources exists')], [('d.json', '{}')])\n"
            "except guard_amd.GuardError as e:\n    print('ERR', e.code, e.message)\n") % os.path.dirname(guard_amd.__file__)
    env = dict(os.environ, GG_DEVICE="999")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert "ERR -1" in r.stdout and "out of range" in r.stdout, r.stdout + r.stderr


def test_reference_validate_resources_vs_oracle():
    """The reference's validate test resources (template without Resources at the root, a key with
    '/', comments, DB port rule, count() with and without messages, malformed / empty inputs) in
    every structured format: byte-identical to the oracle, same exit code; aborting inputs raise."""
    cases = json.load(open(os.path.join(G, "validate_cases.json")))
    for c in cases:
        rules = [tuple(x) for x in c["rules"]]
        data = [tuple(x) for x in c["data"]]
        for fmt in ("json", "yaml", "sarif", "junit"):
            exp, ecode, err = oracle_validate(rules, data, output=fmt)
            if ecode == -1:
                with pytest.raises(guard_amd.GuardError) as ei:
                    guard_amd.validate_structured(rules, data, output=fmt)
                # same abort: the Display the CLI prints after "Error occurred " (main.rs:36-41)
                assert err.endswith("Error occurred " + ei.value.message), (c["source"], fmt)
                continue
            out, code = guard_amd.validate_structured(rules, data, output=fmt)
            assert (code, out) == (ecode, exp), (c["source"], fmt)


def _unicode_docs():
    vals = [("١٢٣", "ñandú-κ", "PROD", "😀"), ("123", "plain_name", "STRASSE", "ab"), ("12 3", "a b", "Straẞe", "é"),
            ("߀߁", "ǅungla", "KELVIN", "😀😀"), ("²", "x½", "ΣΑΣ", ""), ("٣", "日本語", "prod\n", "ſ")]
    docs = []
    for i, (serial, name, env, icon) in enumerate(vals):
        docs.append(json.dumps({"Resources": {
            "r%d" % i: {"Type": "AWS::S3::Bucket" if i % 2 else "AWS::EC2::Volume",
                        "Properties": {"Serial": serial, "Name": name, "Icon": icon,
                                       "Tags": [{"Key": "env", "Value": env}]}}}}, ensure_ascii=False))
    return docs


def test_unicode_regex_pack_vs_oracle():
    """non-ASCII haystacks against \\d \\w \\s (?i) . and anchored alternations, byte-identical with the
    oracle in every format; the DFA tables are LDS-staged (tiny class DFAs)"""
    p = os.path.join(G, "unicode_rulepack")
    rules = [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
    data = [("u%d.json" % i, d) for i, d in enumerate(_unicode_docs())]
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt


def _wordb_docs():
    import random
    r = random.Random(4242)
    names = ["prod-eu", "preprod", "prod", "xprodx", "café", "café-prod", "cafés", "a_b-c", "σοφία prod", "日本 prod",
             "e\u0301-prod", "prod\u0301", "-prod-", ""]
    serials = ["123", "1 2 3", "١٢٣", "12a", "a1", "x", "", "9"]
    icons = ["😀", "a", "é", " ", "_", "-", "σ"]
    envs = ["straße", "STRASSE", "Straße!", "Σοφός", "xσy", "σ", "prod"]
    docs = []
    for i in range(60):
        docs.append(json.dumps({"Resources": {
            "r%d" % k: {"Type": r.choice(["AWS::S3::Bucket", "AWS::EC2::Volume"]),
                        "Properties": {"Name": r.choice(names), "Serial": r.choice(serials), "Icon": r.choice(icons),
                                       "Tags": [{"Key": "env", "Value": r.choice(envs)}]}} for k in range(4)}},
            ensure_ascii=False))
    return docs


def test_word_boundary_regex_pack_vs_oracle():
    """\\b / \\B (Unicode word boundaries) on the device: byte-identical with the oracle in every format,
    lane and wave kernels (tests/golden/wordb_rulepack)"""
    p = os.path.join(G, "wordb_rulepack")
    rules = [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
    data = [("w%d.json" % i, d) for i, d in enumerate(_wordb_docs())]
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt
    s = guard_amd.Session()
    s.configure(1, 0)   # wave mode
    for name, text in rules:
        s.add_rules(text, name)
    s.add_docs([t for _, t in data], [n for n, _ in data])
    s.eval(1)
    exp, ecode, _ = oracle_validate(rules, data)
    assert s.report("json") == (exp, ecode)
    s.close()


def _nfa_docs():
    import random
    r = random.Random(5150)
    cjk = "".join(chr(0x4E00 + 3 * k) for k in range(260))
    docs = []
    for i in range(80):
        res = {}
        for k in range(3):
            n = r.choice([5, 12, 13, 14, 16, 25])
            code = r.choice(["", "c", "q"]) + "".join(r.choice("ab") for _ in range(n))
            props = {"Code": code}
            if r.random() < 0.7:
                m = r.choice([1, 2, 3, 6])
                lab = "".join(r.choice(cjk) for _ in range(m))
                props["Label"] = r.choice([lab, "x" + lab + "y", lab + "!", "ab" + lab])
            res["r%d" % k] = {"Type": "AWS::S3::Bucket", "Properties": props}
        docs.append(json.dumps({"Resources": res}, ensure_ascii=False))
    return docs


def test_nfa_regex_pack_vs_oracle():
    """regexes past the DFA limits run as the NFA simulation on the device (tests/golden/nfa_rulepack):
    byte-identical with the oracle in every format, lane and wave kernels, memo on and off"""
    p = os.path.join(G, "nfa_rulepack")
    rules = [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]
    data = [("n%d.json" % i, d) for i, d in enumerate(_nfa_docs())]
    for fmt in ("json", "sarif"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt
    exp, ecode, _ = oracle_validate(rules, data)
    for mode in (1, 0):
        s = guard_amd.Session()
        s.configure(mode, 0)
        for name, text in rules:
            s.add_rules(text, name)
        s.add_docs([t for _, t in data], [n for n, _ in data])
        s.eval(1)
        assert s.report("json") == (exp, ecode), mode
        s.close()


def test_app_b13_unicode_digit_class_on_gpu():
    rules = [("d.guard", "a == /^\\d+$/")]
    out, code = guard_amd.validate_structured(rules, [("d.json", '{"a": "١٢٣"}')])
    assert code == 0 and '"status": "PASS"' in out


def test_parallel_report_matches_serial():
    """session_report renders contiguous document ranges on host threads and merges them
    (reporter.cpp report_batch); the bytes equal the single-thread rendering in every format"""
    docs = synth.cfn_corpus(700, start=31337, n_resources=20)
    s = guard_amd.Session()
    for name, text in rule_pack():
        s.add_rules(text, name)
    s.add_docs(docs, ["p%d.json" % (i % 500) for i in range(len(docs))])   # repeated names: SARIF dedupe
    s.eval(1)
    try:
        for fmt in ("json", "yaml", "sarif", "junit"):
            os.environ["GG_REPORT_THREADS"] = "1"
            one = s.report(fmt)
            os.environ["GG_REPORT_THREADS"] = "3"
            par = s.report(fmt)
            assert par == one, fmt
            if fmt in ("json", "yaml"):
                os.environ["GG_REPORT_BLOCK"] = "256"   # 3 blocks
                assert s.report_bytes(fmt) == (len(one[0].encode()), one[1]), fmt
    finally:
        os.environ.pop("GG_REPORT_THREADS", None)
        os.environ.pop("GG_REPORT_BLOCK", None)
    s.close()


def test_duplicate_yaml_keys_vs_oracle():
    """a repeated mapping key keeps its first position and takes the last value
    (MapValue.values is an IndexMap, path_value.rs:453-470); value queries over such documents,
    in every output format, against the oracle (its libyaml loader keeps the same first-position /
    last-value mapping; `keys` filters and captures: the test below)."""
    data = [("dup.yaml", "Resources:\n  b:\n    Type: AWS::S3::Bucket\n    Properties:\n      Port: 1\n      Name: x\n"
                         "      Port: 2\n  c:\n    Type: AWS::S3::Bucket\n    Type: AWS::EC2::Volume\n    Properties:\n"
                         "      Size: 300\n")]
    rules = [("dup.guard", "rule ports { Resources.*[ Type == 'AWS::S3::Bucket' ].Properties.Port == 1 }\n"
                           "rule vols { AWS::EC2::Volume { Properties.Size <= 256 } }\n"
                           "rule order { Resources.b.Properties.* exists }\n")]
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt


def _dup_pack():
    p = os.path.join(G, "dupkey_rulepack")
    return [("dup.guard", open(os.path.join(p, "dup.guard")).read())], \
        [("dup.yaml", open(os.path.join(p, "dup.yaml.txt")).read())]


def test_duplicate_keys_keys_filters_and_captures_vs_oracle():
    """SURVEY.md App. B #7 reproduced: MapValue.keys keeps every occurrence of a repeated key
    (loader.rs:172-185) while values keep one entry each (path_value.rs:453-470), so
    * `keys ==` / `keys in` filters compare every occurrence and select values.get(key) once per
      passing occurrence (eval_context.rs:850-880);
    * `Resources[ id ]` / `x[ id | filter ]` captures take accumulate_map's misaligned zip of keys
      with values (eval_context.rs:216);
    * the Debug of such a map (reason R8 / R1 texts) lists the duplicate keys with their marks.
    Byte-identical with the oracle in every format, in lane and wave mode."""
    rules, data = _dup_pack()
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt
    outs = []
    for mode in (0, 1):
        s = guard_amd.Session()
        s.configure(mode, 0)
        s.add_rules(rules[0][1], rules[0][0])
        s.add_docs([data[0][1]] * 70, ["dup.yaml"] * 70)
        s.eval(1)
        outs.append(s.report())
        s.close()
    assert outs[0] == outs[1]


def test_count_result_traversal_vs_oracle():
    """A count() result is an ordinary Int to the query engine: key / index / map-key-filter steps
    on it are UnResolved R8 / R9 / R11 (eval_context.rs:573-581, 587-607, 913-919), `[*]` / `*`
    pass it through (:609-721), a block or a `[*]` filter evaluates over it -- no E_UNSUPPORTED.
    Also the scalar-under-`[*]` filter's clauses are reported with the enclosing clause (no Filter
    container, :790-815).  Every format, lane and wave mode."""
    p = os.path.join(G, "count_rulepack")
    rules = [("cnt.guard", open(os.path.join(p, "cnt.guard")).read())]
    docs = ['{"Resources": {"a": {"Type": "X", "Props": {"Size": 5, "Tags": "t"}}, "b": {"Type": "Y", "Props": {"Size": 50}}}}',
            '{"Other": 1}', '{"Resources": {}}', 'Resources:\n  q:\n    Props:\n      Size: 1\n']
    data = [("t%d.json" % i, d) for i, d in enumerate(docs)]
    for fmt in ("json", "yaml", "sarif", "junit"):
        exp, ecode, _ = oracle_validate(rules, data, output=fmt)
        out, code = guard_amd.validate_structured(rules, data, output=fmt)
        assert (code, out) == (ecode, exp), fmt
    outs = []
    for mode in (0, 1):
        s = guard_amd.Session()
        s.configure(mode, 0)
        s.add_rules(rules[0][1], rules[0][0])
        s.add_docs(docs * 20, ["t%d.json" % (i % 4) for i in range(80)])
        s.eval(1)
        outs.append(s.report())
        s.close()
    assert outs[0] == outs[1]


def test_unreachable_filter_predecessor_panics_like_the_reference():
    """`x[0][ filter ]` on a map: the reference's `_ => unreachable!()` (eval_context.rs:752) panics;
    through guard-ffi that is code -1 with the panic payload, which the device path reports too"""
    rules = [("u.guard", "Resources.list[0][ a exists ] !empty\n")]
    data = [("u.json", '{"Resources": {"list": [{"a": 1}]}}')]
    _, ecode, err = oracle_validate(rules, data)
    assert ecode == -1 and "entered unreachable code" in err
    with pytest.raises(guard_amd.GuardError) as ei:
        guard_amd.validate_structured(rules, data)
    assert ei.value.code == -1 and ei.value.message == "internal error: entered unreachable code"


PARAMS_DIR = os.path.join(G, "params")


def _pfile(rel):
    return (os.path.basename(rel), open(os.path.join(PARAMS_DIR, rel)).read())


# guard/tests/validate.rs:421-473 (test_combinations_of_rules_data_and_input_params_files): -i
# arguments -> the exit code; a directory argument is its sorted supported files (walk_dir)
PARAM_CASES = [
    (["input-parameters-dir/db_params.yaml"], 19),
    (["input-parameters-dir/db_params.yaml", "input-parameters-dir/db_metadata.yaml"], 0),
    (["input-parameters-dir/db_metadata.yaml", "input-parameters-dir/db_params.yaml"], 0),   # "input-parameters-dir/"
    (["malformed-template.yaml"], -1),
    (["blank-template.yaml"], -1),
    (["blank-template.yaml", "input-parameters-dir/db_params.yaml"], -1),
]


def test_input_parameters_reference_cases():
    """validate -i (validate.rs:317-350, structured.rs:51-65, path_value.rs:889-919): the six cases of
    guard/tests/validate.rs:421-473 give the reference's exit codes, with byte parity vs the oracle
    in every format and the same abort (code + message) where the run aborts"""
    rules = [_pfile("db_param_port_rule.guard")]
    data = [_pfile("db_resource.yaml")]
    for files, want in PARAM_CASES:
        params = [_pfile(f) for f in files]
        for fmt in ("json", "yaml", "sarif", "junit"):
            exp, ecode, err = oracle_validate(rules, data, output=fmt, params=params)
            assert ecode == want, (files, fmt)
            if want == -1:
                with pytest.raises(guard_amd.GuardError) as ei:
                    guard_amd.validate_structured(rules, data, output=fmt, params=params)
                assert err == "Error occurred " + ei.value.message, files
                continue
            out, code = guard_amd.validate_structured(rules, data, output=fmt, params=params)
            assert (code, out) == (ecode, exp), (files, fmt)


def test_input_parameters_merge_semantics_vs_oracle():
    """merged roots: self's (the parameters') location, self's keys then other's keys at other's
    path + "/key" and location (path_value.rs:905-907) -- seen through root captures and R7 / Display
    of the merged root; a repeated key in a parameter file (key block kept through the merge); list
    roots concatenate with every element keeping its own path.  Every format, lane and wave mode."""
    rules = [_pfile("params_keys.guard")]
    data = [_pfile("db_resource.yaml")]
    for files in (["input-parameters-dir/db_params.yaml", "input-parameters-dir/db_metadata.yaml"], ["dup_params.yaml"]):
        params = [_pfile(f) for f in files]
        for fmt in ("json", "yaml", "sarif", "junit"):
            exp, ecode, _ = oracle_validate(rules, data, output=fmt, params=params)
            out, code = guard_amd.validate_structured(rules, data, output=fmt, params=params)
            assert (code, out) == (ecode, exp), (files, fmt)
        outs = []
        for mode in (0, 1):
            s = guard_amd.Session()
            s.configure(mode, 0)
            s.add_rules(rules[0][1], rules[0][0])
            s.set_params(params)
            s.add_docs([data[0][1]] * 70, ["db-%d.yaml" % i for i in range(70)])
            s.eval(1)
            outs.append(s.report())
            s.close()
        assert outs[0] == outs[1]
    lrules = [("l.guard", "this[*] > 5\nthis[3] == 1\n")]
    ldata = [("l.yaml", "- 1\n- 2\n")]
    lparams = [("p.yaml", "- 7\n- 3\n")]
    exp, ecode, _ = oracle_validate(lrules, ldata, params=lparams)
    out, code = guard_amd.validate_structured(lrules, ldata, params=lparams)
    assert (code, out) == (ecode, exp)


def test_input_parameters_conflicts_abort_like_the_reference():
    """between parameter files a merge error propagates (MultipleValues 9 / IncompatibleError 11);
    between the parameters and a data file the reference unwraps the merge and panics (code -1)"""
    rules = [_pfile("db_param_port_rule.guard")]
    data = [_pfile("db_resource.yaml")]
    cases = [([("p.yaml", "Resources: {}\n")], -1),
             ([("p.yaml", "- 1\n")], -1),
             ([("p.yaml", "a: 1\n"), ("q.yaml", "a: 2\n")], 9),
             ([("p.yaml", "a: 1\n"), ("q.yaml", "- 2\n")], 11)]
    for params, code in cases:
        _, ecode, err = oracle_validate(rules, data, params=params)
        assert ecode == -1
        with pytest.raises(guard_amd.GuardError) as ei:
            guard_amd.validate_structured(rules, data, params=params)
        assert ei.value.code == code and err == "Error occurred " + ei.value.message, params
