"""Structured output formats other than JSON (TEST INFRASTRUCTURE ONLY -- the parity oracle).

* YAML: ``serde_yaml::to_writer(&records)`` (``reporters/validate/structured.rs:126``).
  serde_yaml 0.9 drives unsafe-libyaml (a port of libyaml 0.2.5) with line width unlimited; a
  string is emitted in literal style when it contains a newline, single-quoted when its plain
  form would resolve to a non-string (null / bool / int / float, YAML 1.2 core schema) and in
  the emitter's own choice of style otherwise.  The same libyaml emitter runs here through
  PyYAML's C binding, fed the event stream serde_yaml produces.
* SARIF: ``SarifReport::new`` (``reporters/validate/sarif.rs``) through serde_json's pretty writer.
* JUnit: ``JunitReporter::report`` (``reporters/validate/xml.rs``) and the quick_xml writer of
  ``reporters/mod.rs:66-420`` (indent 4, attribute / text escaping of ``<>&'"``).

All three are pinned byte-for-byte by guard/resources/validate/output-dir/structured.{yaml,sarif,junit}.
"""
import io
import re

import yaml

from . import pv as P
from .report import OMap, Msgs, to_json_pretty

# --------------------------------------------------------------------------------------- YAML
_NULL = {"~", "null", "Null", "NULL"}
_BOOL = {"true", "True", "TRUE", "false", "False", "FALSE"}
# serde_yaml de.rs parse_unsigned_int / parse_negative_int (radix prefixes; decimal runs of digits
# are covered by the float grammar, which Rust's f64 parser accepts for any digit string)
_INT = re.compile(r"^\+?0x[0-9a-fA-F]+$|^\+?0o[0-7]+$|^\+?0b[01]+$|^-0x[0-9a-fA-F]+$|^-0o[0-7]+$|^-0b[01]+$")
# parse_f64: optional sign, Rust f64 grammar, finite values only; .inf / .nan spellings
_FLOAT = re.compile(r"^[-+]?(\.[0-9]+|[0-9]+(\.[0-9]*)?)([eE][-+]?[0-9]+)?$")
_SPECIAL = re.compile(r"^[-+]?\.(inf|Inf|INF)$|^\.(nan|NaN|NAN)$")


def _resolves_to_non_string(v):
    """serde_yaml de::visit_untagged_scalar over the plain form: empty / null, bool, int, float"""
    if v == "" or v in _NULL or v in _BOOL:
        return True
    if v.startswith("+") and v[1:2] in ("+", "-"):
        return False
    if _INT.match(v) or _SPECIAL.match(v):
        return True
    if _FLOAT.match(v):
        return float(v) not in (float("inf"), float("-inf"))
    return False


def _str_style(v):
    if "\n" in v:
        return "|"
    return "'" if _resolves_to_non_string(v) else None


def _yaml_float(x):
    if x != x:
        return ".nan"
    if x in (float("inf"), float("-inf")):
        return ".inf" if x > 0 else "-.inf"
    return P.ryu_f64(x)


def _scalar(value, style=None):
    return yaml.ScalarEvent(None, None, (True, True), value, style=style)


def _yaml_events(o, out):
    if o is None:
        out.append(_scalar("null"))
    elif o is True or o is False:
        out.append(_scalar("true" if o else "false"))
    elif isinstance(o, P.JFloat):
        out.append(_scalar(_yaml_float(o.v)))
    elif isinstance(o, int):
        out.append(_scalar(str(o)))
    elif isinstance(o, str):
        out.append(_scalar(o, _str_style(o)))
    elif isinstance(o, (OMap, dict)):
        items = o.items if isinstance(o, OMap) else list(o.items())
        out.append(yaml.MappingStartEvent(None, None, True, flow_style=False))
        for k, v in items:
            out.append(_scalar(k, _str_style(k)))
            _yaml_events(v, out)
        out.append(yaml.MappingEndEvent())
    elif isinstance(o, (list, tuple)):
        out.append(yaml.SequenceStartEvent(None, None, True, flow_style=False))
        for v in o:
            _yaml_events(v, out)
        out.append(yaml.SequenceEndEvent())
    else:
        raise TypeError(type(o))


def to_yaml(records):
    events = [yaml.StreamStartEvent(), yaml.DocumentStartEvent(explicit=False)]
    _yaml_events(records, events)
    events += [yaml.DocumentEndEvent(explicit=False), yaml.StreamEndEvent()]
    buf = io.StringIO()
    yaml.emit(events, buf, Dumper=yaml.CDumper, width=-1, allow_unicode=True)
    return buf.getvalue()


# -------------------------------------------------------------------------------------- SARIF
SARIF_DRIVER = OMap([
    ("name", "cfn-guard"), ("semanticVersion", "3.1.2"), ("fullName", "cfn-guard 3.1.2"),
    ("organization", "Amazon Web Services"),
    ("downloadUri", "https://github.com/aws-cloudformation/cloudformation-guard"),
    ("informationUri", "https://github.com/aws-cloudformation/cloudformation-guard"),
    ("shortDescription", OMap([("text", "AWS CloudFormation Guard is an open-source general-purpose policy-as-code "
                                        "evaluation tool. It provides developers with a simple-to-use, yet powerful and "
                                        "expressive domain-specific language (DSL) to define policies and enables "
                                        "developers to validate JSON- or YAML- formatted structured data with those "
                                        "policies.")])),
])


def _field(o, k):
    for kk, v in o.items:
        if kk == k:
            return v
    return None


def get_message(clause):
    """ClauseReport::get_message (eval_context.rs:1808-1826)"""
    (kind, body), = clause.items
    if kind in ("Rule", "Disjunctions"):
        out = []
        for ch in _field(body, "checks"):
            out.extend(get_message(ch))
        return out
    if kind == "Block":
        return [_field(body, "messages")]
    (_, inner), = body.items
    return [_field(inner, "messages")]


def _sanitize(path):
    return path[1:] if path.startswith("/") else path


def to_sarif(records):
    artifacts, seen, results = [], set(), []
    for rep in records:
        if _field(rep, "status") != "FAIL":
            continue
        name = _field(rep, "name")
        if name not in seen and name:
            seen.add(name)
            artifacts.append(OMap([("location", OMap([("uri", _sanitize(name))]))]))
        for failure in _field(rep, "not_compliant"):
            (kind, body), = failure.items
            rule_id = _field(body, "name").split(".")[0].upper() if kind == "Rule" else ""
            for m in get_message(failure):
                loc = m.location if isinstance(m, Msgs) and m.location is not None else (0, 0)
                text = "%s %s" % (_field(m, "error_message") or "", _field(m, "custom_message") or "")
                results.append(OMap([
                    ("ruleId", rule_id), ("level", "error"), ("message", OMap([("text", text)])),
                    ("locations", [OMap([("physicalLocation", OMap([
                        ("artifactLocation", OMap([("uri", _sanitize(name))])),
                        ("region", OMap([("startLine", max(loc[0], 1)), ("startColumn", max(loc[1], 1))]))]))])])]))
    run = OMap([("tool", OMap([("driver", SARIF_DRIVER)])), ("artifacts", artifacts), ("results", results)])
    return to_json_pretty(OMap([
        ("$schema", "https://docs.oasis-open.org/sarif/sarif/v2.1.0/errata01/os/schemas/sarif-schema-2.1.0.json"),
        ("version", "2.1.0"), ("runs", [run])]))


# -------------------------------------------------------------------------------------- JUnit
def _xml_escape(s):
    return (s.replace("&", "&amp;").replace("<", "&lt;").replace(">", "&gt;")
            .replace("'", "&apos;").replace('"', "&quot;"))


def junit_test_case(rules_name, status, report):
    """get_test_case (reporters/mod.rs:108-168): (name, status, failure name, failure texts)"""
    if status != "FAIL":
        return (rules_name, "pass" if status == "PASS" else "skip", None, None)
    fname, texts = None, []
    for failure in report["not_compliant"]:
        (kind, body), = failure.items
        for m in get_message(failure):
            if kind == "Rule":
                rn = _field(body, "name")
                fname = rn.split(".guard/")[1] if ".guard/" in rn else rn
            if _field(m, "custom_message") is not None:
                texts.append(_field(m, "custom_message"))
            if _field(m, "error_message") is not None:
                texts.append(_field(m, "error_message"))
    return (rules_name, "fail", fname, texts)


def to_junit(suites):
    """suites: [(data_name, [test cases from junit_test_case])] -> quick_xml text"""
    tests = sum(len(tc) for _, tc in suites)
    failures = sum(1 for _, tc in suites for c in tc if c[1] == "fail")
    out = ['<?xml version="1.0" encoding="UTF-8"?>',
           '<testsuites name="cfn-guard validate report" tests="%d" failures="%d" errors="0" time="0">' % (tests, failures)]
    for name, cases in suites:
        nf = sum(1 for c in cases if c[1] == "fail")
        out.append('    <testsuite name="%s" errors="0" failures="%d" time="0">' % (_xml_escape(name), nf))
        for rname, st, fname, texts in cases:
            if st != "fail":
                out.append('        <testcase name="%s" time="0" status="%s"/>' % (_xml_escape(rname), st))
                continue
            out.append('        <testcase name="%s" time="0">' % _xml_escape(rname))
            attr = ' message="%s"' % _xml_escape(fname) if fname is not None else ""
            if texts:
                out.append('            <failure%s>%s</failure>' % (attr, "".join(_xml_escape(t) for t in texts)))
            else:
                out.append('            <failure%s/>' % attr)
            out.append('        </testcase>')
        out.append('    </testsuite>')
    out.append('</testsuites>')
    return "\n".join(out) + "\n"
