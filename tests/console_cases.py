"""Console (non-structured) `cfn-guard validate` cases pinned by the reference's own tests
(guard/tests/validate.rs:237-345, 405-418, 488-540) and their golden outputs
(guard/resources/validate/output-dir/*.out and functions/output/*.out, copied to
tests/golden/validate/output-dir and tests/golden/validate/functions/output).

Each case: (name, rules [(name, text)], data [(name, text)], options, expected stdout, exit code,
needs look-around).  expected None: the reference test asserts the exit code only.
Data names are the file names the tests' sanitize_path leaves of the CLI's canonical paths
(tests/utils.rs:130-150); data read from stdin is named STDIN (validate.rs:303-312)."""
import json
import os

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "validate")
OUT = os.path.join(GOLD, "output-dir")


def _read(*p):
    with open(os.path.join(GOLD, *p)) as f:
        return f.read()


def _data(*names):
    out = []
    for n in names:
        p = n if "/" in n else n
        out.append((os.path.basename(n), _read(*p.split("/"))))
    return out


def _rules(*names):
    return [(os.path.basename(n), _read(*n.split("/"))) for n in names]


def _stdin(name):
    return [("STDIN", _read("data-dir", name))]


def _out(name):
    with open(os.path.join(OUT, name)) as f:
        return f.read()


COMPLIANT_SUMMARY = (
    "s3-public-read-prohibited-template-compliant.yaml Status = PASS\n"
    "PASS rules\n"
    "s3_bucket_public_read_prohibited.guard/S3_BUCKET_PUBLIC_READ_PROHIBITED    PASS\n"
    "---\n")


def _dir(sub, exts):
    return sorted(f for f in os.listdir(os.path.join(GOLD, sub)) if f.endswith(exts))


def cases():
    """(name, rules, data, opts, expected, code, needs_lookaround)"""
    pr = "rules-dir/s3_bucket_public_read_prohibited.guard"
    sse = "rules-dir/s3_bucket_server_side_encryption_enabled.guard"
    rx = "rules-dir/advanced_regex_negative_lookbehind_rule.guard"
    all_ = {"summary": ("all",)}
    allv = {"summary": ("all",), "verbose": True}
    c = [
        ("compliant_summary_all", _rules(pr), _data("data-dir/s3-public-read-prohibited-template-compliant.yaml"),
         all_, COMPLIANT_SUMMARY, 0, False),
        ("verbose_compliant", _rules(pr), _data("data-dir/s3-public-read-prohibited-template-compliant.yaml"), allv,
         _out("test_single_data_file_single_rules_file_verbose_compliant.out"), 0, False),
        ("verbose_non_compliant", _rules(pr), _data("data-dir/s3-public-read-prohibited-template-non-compliant.yaml"),
         allv, _out("test_single_data_file_single_rules_file_verbose_non_compliant.out"), 19, False),
        ("resources_not_at_root", _rules("workshop.guard"), _data("template_where_resources_isnt_root.json"), allv,
         _out("failing_template_without_resources_at_root.out"), 19, False),
        ("slash_in_key", _rules(sse), _data("failing_template_with_slash_in_key.yaml"), allv,
         _out("failing_template_with_slash_in_key.out"), 19, False),
        ("non_compliant_summary_all", _rules(pr), _data("data-dir/s3-public-read-prohibited-template-non-compliant.yaml"),
         all_, _out("test_single_data_file_single_rules_file_verbose.out"), 19, False),
        ("lookbehind_non_compliant", _rules(rx), _data("data-dir/advanced_regex_negative_lookbehind_non_compliant.yaml"),
         all_, _out("advanced_regex_negative_lookbehind_non_compliant.out"), 19, True),
        ("lookbehind_compliant", _rules(rx), _data("data-dir/advanced_regex_negative_lookbehind_compliant.yaml"),
         all_, _out("advanced_regex_negative_lookbehind_compliant.out"), 0, True),
        ("rules_dir_against_data_dir", _rules(*["rules-dir/" + f for f in _dir("rules-dir", (".guard", ".ruleset"))]),
         _data(*["data-dir/" + f for f in _dir("data-dir", (".yaml", ".yml", ".json", ".jsn", ".template"))]),
         {}, _out("rules_dir_against_data_dir.out"), 19, True),
        ("stdin_verbose_success", _rules(pr), _stdin("s3-server-side-encryption-template-compliant.yaml"),
         {"verbose": True}, _out("payload_verbose_success.out"), 0, False),
        ("stdin_verbose_fail", _rules(pr), _stdin("s3-public-read-prohibited-template-non-compliant.yaml"),
         {"verbose": True}, _out("payload_verbose_non_compliant.out"), 19, False),
        ("stdin_verbose_yaml", _rules(pr), _stdin("s3-public-read-prohibited-template-compliant.yaml"),
         {"verbose": True, "output": "yaml"}, _out("payload_verbose_yaml_compliant.out"), 0, False),
        # validate.rs:733-749: a count() over an unresolved query compared with a literal
        ("failing_count_show_summary_all", _fn_rules("count_with_message.guard"), _fn_data(), all_,
         _fn_out("failing_count_show_summary_all.out"), 19, False),
        # validate.rs:709-731 (the count() member of test_validate_with_fn_expr_success)
        ("fn_expr_success_count", _fn_rules("count.guard"), _fn_data(), allv, None, 0, False),
        # validate.rs:566-597: --payload, data / rules named DATA_STDIN[i] / RULES_STDIN[i]
        ("payload_flag_fail", *_payload(PAYLOAD_FAIL), {}, PAYLOAD_FAIL_OUT, 19, False),
        ("payload_flag", *_payload(PAYLOAD_OK), {}, None, 0, False),
    ]
    # validate.rs:788-807: rules-dir against a non-compliant S3 template (the look-behind rule's
    # queries resolve nothing there, so its regexes are never evaluated)
    for ss in (("pass", "fail"), ("skip", "fail"), ("skip", "pass")):
        c.append(("show_summary_" + "_".join(ss),
                  _rules(*["rules-dir/" + f for f in _dir("rules-dir", (".guard", ".ruleset"))]),
                  _data("data-dir/s3-public-read-prohibited-template-non-compliant.yaml"),
                  {"summary": ss}, None, 19, False))
    return c


FN = os.path.join(GOLD, "functions")


def _fn_rules(*names):
    out = []
    for n in names:
        with open(os.path.join(FN, "rules", n)) as f:
            out.append((n, f.read()))
    return out


def _fn_data():
    with open(os.path.join(FN, "data", "template.yaml")) as f:
        return [("template.yaml", f.read())]


def _fn_out(name):
    with open(os.path.join(FN, "output", name)) as f:
        return f.read()


def _payload(text):
    """validate.rs:438-464: the payload's data / rules strings, named by position"""
    p = json.loads(text)
    return ([("RULES_STDIN[%d]" % (i + 1), r) for i, r in enumerate(p["rules"])],
            [("DATA_STDIN[%d]" % (i + 1), d) for i, d in enumerate(p["data"])])


# validate.rs:568, 584: both payloads carry this document twice
_VOL = ('{"Resources":{"NewVolume":{"Type":"AWS::EC2::Volume","Properties":{"Size":500,"Encrypted":false,'
        '"AvailabilityZone":"us-west-2b"}},"NewVolume2":{"Type":"AWS::EC2::Volume","Properties":{"Size":50,'
        '"Encrypted":false,"AvailabilityZone":"us-west-2c"}}},"Parameters":{"InstanceName":"TestInstance"}}')
PAYLOAD_OK = json.dumps({"data": [_VOL, _VOL], "rules": ['Parameters.InstanceName == "TestInstance"'] * 2})
PAYLOAD_FAIL = json.dumps({"data": [_VOL, _VOL], "rules": ['Parameters.InstanceName == "TestInstance"',
                                                           'Parameters.InstanceName == "SomeRandomString"']})
PAYLOAD_FAIL_OUT = "".join(
    "DATA_STDIN[%d] Status = FAIL\n"
    "FAILED rules\n"
    "RULES_STDIN[2]/default    FAIL\n"
    "---\n"
    "Evaluating data DATA_STDIN[%d] against rules RULES_STDIN[2]\n"
    "Number of non-compliant resources 0\n" % (i, i) for i in (1, 2))
# validate.rs:555-564: a type block over a query that resolves nothing -> an evaluation error (exit -1)
PAYLOAD_TYPE_BLOCK = json.dumps({"data": ["{}"], "rules": ["d1z::Y\n\t\tm<0m<03333333"]})
