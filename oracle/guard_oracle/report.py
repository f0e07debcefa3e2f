"""Structured report restatement (TEST INFRASTRUCTURE ONLY -- the parity oracle).

Restates ``report_all_failed_clauses_for_rules`` / ``simplified_json_from_root``
(``guard/src/rules/eval_context.rs:1965-2435``), ``FileReport::combine`` (:1630-1640),
the structured loop ``CommonStructuredReporter::report``
(``commands/reporters/validate/structured.rs:99-133``) and serde_json's pretty writer
(``to_writer_pretty``: 2-space indent, ryu floats, struct field order = declaration order).
"""
from .errors import GuardError
from . import pv as P
from .parser import slice_display, parse_rules
from . import evaluator as E
from .loader import load_document

CMP_NAME = {k: k for k in ("Eq", "In", "Gt", "Lt", "Le", "Ge", "Exists", "Empty", "IsString", "IsList",
                            "IsMap", "IsBool", "IsInt", "IsFloat", "IsNull")}


class OMap:
    """ordered JSON object (serde struct / IndexMap)"""
    __slots__ = ("items",)

    def __init__(self, items):
        self.items = items


class PavJ(OMap):
    """a serialized PathAwareValue that keeps the value itself (the console reporters read its
    location and ValueOnlyDisplay, commands/reporters/validate/cfn.rs)"""
    __slots__ = ("pv",)

    def __init__(self, items, pv):
        OMap.__init__(self, items)
        self.pv = pv


class UrJ(PavJ):
    __slots__ = ("ur",)


def _ur_json(ur):
    o = UrJ([("traversed_to", P.serialize(ur.traversed_to)),
             ("remaining_query", ur.remaining_query),
             ("reason", ur.reason)], ur.traversed_to)
    o.ur = ur
    return o


def _pav_json(v):
    s = P.serialize(v)
    return PavJ([("path", s["path"]), ("value", s["value"])], v)


class Msgs(OMap):
    """Messages (eval_context.rs:1608-1614): custom_message, error_message; ``location`` is
    skip_serializing but read by the SARIF writer (sarif.rs:139-142)"""
    __slots__ = ("location",)

    def __init__(self, items, location=None):
        OMap.__init__(self, items)
        self.location = location


def _loc(v):
    return (v.line, v.col)


def _messages(custom, error, location=None):
    return Msgs([("custom_message", custom), ("error_message", error)], location)


def _unary_cmp_msg(cmp, neg):
    table = {
        "Exists": ("existed", "did not exist"), "Empty": ("was empty", "was not empty"),
        "IsList": ("was a list ", "was not list"), "IsMap": ("was a struct", "was not struct"),
        "IsString": ("was a string ", "was not string"), "IsInt": ("was int", "was not int"),
        "IsBool": ("was bool", "was not bool"), "IsNull": ("was null", "was not null"),
    }
    a, b = table.get(cmp, ("was float", "was not float"))
    return a if neg else b


_OP_MSG = {
    "Eq": ("equal to", "not equal to"), "Le": ("less than equal to", "not less than equal to"),
    "Lt": ("less than", "not less than"), "Ge": ("greater than equal to", "not greater than equal"),
    "Gt": ("greater than", "not greater than"), "In": ("in", "not in"),
}


def _qr_display(q):
    # impl Display for QueryResult (display.rs:109-126)
    k, v = q
    if k == "L":
        return "literal, %s" % P.display(v)
    if k == "R":
        return "(resolved, %s)" % P.display(v)
    return "(unresolved, %s)" % P.display(v.traversed_to)


def report_all_failed(checks):
    clauses = []
    for cur in checks:
        c = cur.container
        if c is None:
            continue
        k = c[0]
        if k == "RuleCheck" and c[2] == E.FAIL:
            clauses.append(("Rule", OMap([
                ("name", c[1]), ("metadata", OMap([])),
                ("messages", _messages(c[3], None)),
                ("checks", report_all_failed(cur.children))])))
        elif k == "BlockGuardCheck" and c[1] == E.FAIL:
            if not cur.children:
                clauses.append(("Block", OMap([
                    ("context", cur.context),
                    ("messages", _messages(None, "query for block clause did not retrieve any value")),
                    ("unresolved", None)])))
            else:
                clauses.extend(report_all_failed(cur.children))
        elif k == "Disjunction" and c[1] == E.FAIL:
            clauses.append(("Disjunctions", OMap([("checks", report_all_failed(cur.children))])))
        elif k in ("GuardClauseBlockCheck", "TypeBlock", "TypeCheck", "WhenCheck") and c[1] == E.FAIL:
            clauses.extend(report_all_failed(cur.children))
        elif k == "ClauseValueCheck":
            cc = c[1]
            ck = cc[0]
            if ck == "NoValueForEmptyCheck":
                custom = (cc[1] or "").replace("\n", ";")
                err = "Check was not compliant as variable in context [%s] was not empty" % cur.context
                clauses.append(("Clause", ("Unary", OMap([
                    ("check", OMap([("UnResolvedContext", cur.context)])),
                    ("context", cur.context),
                    ("messages", _messages(custom, err))]))))
            elif ck == "DependentRule":
                m = cc[1]
                err = "Check was not compliant as dependent rule [%s] did not PASS. Context [%s]" % (m["rule"], cur.context)
                clauses.append(("Clause", ("Unary", OMap([
                    ("check", OMap([("UnResolvedContext", m["rule"])])),
                    ("context", cur.context),
                    ("messages", _messages(m["custom_message"] or "", err))]))))
            elif ck == "MissingBlockValue":
                m = cc[1]
                ur = m["from"][1]
                err = "Check was not compliant as property [%s] is missing. Value traversed to [%s]" % (
                    ur.remaining_query, P.display(ur.traversed_to))
                clauses.append(("Block", OMap([
                    ("context", cur.context),
                    ("messages", _messages(m["custom_message"] or "", err)),
                    ("unresolved", _ur_json(ur))])))
            elif ck == "Unary":
                m = cc[1]
                cmp, neg = m["comparison"]
                cmp_msg = _unary_cmp_msg(cmp, neg)
                custom = m["custom_message"] or ""
                errm = "" if m["message"] is None else "Error = [%s]" % m["message"]
                frm = m["from"]
                if frm[0] == "R":
                    res = frm[1]
                    msg = "Check was not compliant as property [%s] %s.%s" % (res.path_display(), cmp_msg, errm)
                    check = OMap([("Resolved", OMap([("value", _pav_json(res)), ("comparison", [cmp, neg])]))])
                    loc = (0, 0)   # Location::default() (eval_context.rs:2231-2234)
                else:
                    ur = frm[1]
                    msg = "Check was not compliant as property [%s] is missing. Value traversed to [%s].%s" % (
                        ur.remaining_query, P.display(ur.traversed_to), errm)
                    check = OMap([("UnResolved", OMap([("value", _ur_json(ur)), ("comparison", [cmp, neg])]))])
                    loc = _loc(ur.traversed_to)
                clauses.append(("Clause", ("Unary", OMap([
                    ("check", check), ("context", cur.context), ("messages", _messages(custom, msg, loc))]))))
            elif ck == "Comparison":
                m = cc[1]
                cmp, neg = m["comparison"]
                custom = m["custom_message"] or ""
                errm = "" if m["message"] is None else " Error = [%s]" % m["message"]
                frm = m["from"]
                if frm[0] == "U":
                    ur = frm[1]
                    msg = ("Check was not compliant as property [%s] to compare from is missing. "
                           "Value traversed to [%s].%s" % (ur.remaining_query, P.display(ur.traversed_to), errm))
                    clauses.append(("Clause", ("Binary", OMap([
                        ("context", cur.context), ("messages", _messages(custom, msg, _loc(ur.traversed_to))),
                        ("check", OMap([("UnResolved", OMap([("value", _ur_json(ur)), ("comparison", [cmp, neg])]))]))]))))
                else:
                    res = frm[1]
                    to = m["to"]
                    if to is None:
                        continue
                    if to[0] == "R":
                        a, b = _OP_MSG[cmp]
                        msg = "Check was not compliant as property value [%s] %s value [%s].%s" % (
                            P.display(res), a if neg else b, P.display(to[1]), errm)
                        clauses.append(("Clause", ("Binary", OMap([
                            ("context", cur.context), ("messages", _messages(custom, msg, _loc(to[1]))),
                            ("check", OMap([("Resolved", OMap([("from", _pav_json(res)), ("to", _pav_json(to[1])),
                                                               ("comparison", [cmp, neg])]))]))]))))
                    else:
                        ur = to[1]
                        msg = ("Check was not compliant as property [%s] to compare to is missing. "
                               "Value traversed to [%s].%s" % (ur.remaining_query, P.display(ur.traversed_to), errm))
                        clauses.append(("Clause", ("Binary", OMap([
                            ("context", cur.context), ("messages", _messages(custom, msg, _loc(ur.traversed_to))),
                            ("check", OMap([("UnResolved", OMap([("value", _ur_json(ur)), ("comparison", [cmp, neg])]))]))]))))
            elif ck == "InComparison":
                m = cc[1]
                frm = m["from"][1]
                to = m["to"]
                err = "Check was not compliant as property [%s] was not present in [%s]" % (
                    frm.path_display(), slice_display(to, _qr_display))
                clauses.append(("Clause", ("Binary", OMap([
                    ("context", cur.context),
                    ("messages", _messages(m["custom_message"], err, _loc(frm))),
                    ("check", OMap([("InResolved", OMap([
                        ("from", _pav_json(frm)),
                        ("to", [_pav_json(t[1]) for t in to if t[0] == "R"]),
                        ("comparison", list(m["comparison"]))]))]))]))))
    return clauses


def _clause_json(c):
    kind, body = c
    if kind == "Clause":
        sub, inner = body
        return OMap([("Clause", OMap([(sub, _fix(inner))]))])
    return OMap([(kind, _fix(body))])


def _fix(o):
    if isinstance(o, Msgs):
        return Msgs([(k, _fix(v)) for k, v in o.items], o.location)
    if isinstance(o, OMap):
        return OMap([(k, _fix(v)) for k, v in o.items])
    if isinstance(o, list):
        return [_fix_item(x) for x in o]
    return o


def _fix_item(x):
    if isinstance(x, tuple) and len(x) == 2 and isinstance(x[0], str) and x[0] in (
            "Rule", "Block", "Disjunctions", "Clause"):
        return _clause_json(x)
    return _fix(x)


def simplified_json_from_root(root):
    c = root.container
    assert c[0] == "FileCheck"
    passed, skipped = set(), set()
    for ch in root.children:
        cc = ch.container
        if cc is not None and cc[0] == "RuleCheck":
            if cc[2] == E.PASS:
                passed.add(cc[1])
            elif cc[2] == E.SKIP:
                skipped.add(cc[1])
    return {"name": c[1], "status": c[2], "not_compliant": report_all_failed(root.children),
            "not_applicable": skipped, "compliant": passed}


def _rust_str_key(s):
    return s.encode("utf-8", "surrogatepass")


def file_report_json(fr):
    return OMap([("name", fr["name"]), ("metadata", OMap([])), ("status", fr["status"]),
                 ("not_compliant", [_clause_json(c) for c in fr["not_compliant"]]),
                 ("not_applicable", sorted(fr["not_applicable"], key=_rust_str_key)),
                 ("compliant", sorted(fr["compliant"], key=_rust_str_key))])


# ---------------------------------------------------------------------------
# serde_json pretty writer
# ---------------------------------------------------------------------------
def _json_str(s):
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\f":
            out.append("\\f")
        elif o < 0x20:
            out.append("\\u%04x" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def to_json_pretty(o, indent=0):
    pad = "  " * indent
    pad1 = "  " * (indent + 1)
    if o is None:
        return "null"
    if o is True:
        return "true"
    if o is False:
        return "false"
    if isinstance(o, P.JFloat):
        return P.ryu_f64(o.v)
    if isinstance(o, int):
        return str(o)
    if isinstance(o, str):
        return _json_str(o)
    if isinstance(o, OMap):
        if not o.items:
            return "{}"
        parts = ["%s%s: %s" % (pad1, _json_str(k), to_json_pretty(v, indent + 1)) for k, v in o.items]
        return "{\n" + ",\n".join(parts) + "\n" + pad + "}"
    if isinstance(o, dict):
        return to_json_pretty(OMap(list(o.items())), indent)
    if isinstance(o, (list, tuple)):
        if not o:
            return "[]"
        parts = ["%s%s" % (pad1, to_json_pretty(v, indent + 1)) for v in o]
        return "[\n" + ",\n".join(parts) + "\n" + pad + "]"
    raise TypeError(type(o))


# ---------------------------------------------------------------------------
# drivers
# ---------------------------------------------------------------------------
SUCCESS, FAILURE_STATUS, ERROR_STATUS = 0, 19, 5


def eval_file_report(rules_file, doc, data_name):
    root = E.RootScope(rules_file, doc)
    status = E.eval_rules_file(rules_file, root, data_name)
    rec = root.recorder.final_event
    return status, simplified_json_from_root(rec)


def validate_structured(rules, data, parsed_docs=None, output="json", raise_errors=False, params=None):
    """``cfn-guard validate --structured -o {json|yaml|sarif|junit} -S none [-i ...]`` over in-memory inputs.

    rules: list of (rules_file_name, text); data: list of (data_name, text); params: input
    parameter files (name, text) in the CLI's walk order (validate.rs:317-350).
    Returns (stdout_text, exit_code, stderr_text).  Evaluation errors abort the run with
    no stdout, exit code -1 (main.rs:35-42); raise_errors=True re-raises the GuardError instead
    (its kind gives the guard-ffi code, errors.rs:12-38)."""
    exit_code = SUCCESS
    stderr = []
    parsed_rules = []
    for name, text in rules:
        try:
            rf = parse_rules(text, name)
        except GuardError as e:
            stderr.append("Parsing error handling rule file = %s, Error = %s\n---" % (name, e.display()))
            exit_code = ERROR_STATUS
            continue
        if rf is not None:
            parsed_rules.append((rf, name))
    try:
        docs = parsed_docs if parsed_docs is not None else [(n, load_document(t, n)) for n, t in data]
        if params:
            # validate.rs:317-350: every parameter file loaded like a data file, merged in order
            # (`primary.merge(path_value)?`: an error aborts)
            from .pv import merge as pv_merge, rust_debug_str
            primary = None
            for n, t in params:
                pv = load_document(t, n)
                primary = pv if primary is None else pv_merge(primary, pv)
            # structured.rs:51-65: `data.clone().merge(file.path_value.clone()).unwrap()` -- a panic
            merged = []
            for n, doc in docs:
                try:
                    merged.append((n, pv_merge(primary, doc)))
                except GuardError as e:
                    raise GuardError("Panic", "called `Result::unwrap()` on an `Err` value: %s(%s)"
                                     % (e.kind, rust_debug_str(e.msg)))
            docs = merged
        from . import formats
        records, suites = [], []
        for dname, doc in docs:
            fr = {"name": dname, "status": E.SKIP, "not_compliant": [], "not_applicable": set(), "compliant": set()}
            cases = []
            for rf, rname in parsed_rules:
                st, rep = eval_file_report(rf, doc, dname)
                # CommonStructuredReporter sets 19 over a parse error's 5 (structured.rs:110-112);
                # JunitReporter::update_exit_code keeps 5 (reporters/mod.rs:97-103, xml.rs:62-66)
                if st == E.FAIL and not (output == "junit" and exit_code == ERROR_STATUS):
                    exit_code = FAILURE_STATUS
                fr["status"] = E.status_and(fr["status"], rep["status"])
                fr["not_compliant"].extend(rep["not_compliant"])
                fr["compliant"] |= rep["compliant"]
                fr["not_applicable"] |= rep["not_applicable"]
                if output == "junit":
                    cases.append(formats.junit_test_case(
                        rname, st, {"not_compliant": [_clause_json(c) for c in rep["not_compliant"]]}))
            records.append(file_report_json(fr))
            suites.append((dname, cases))
        if output == "json":
            out = to_json_pretty(records)
        elif output == "yaml":
            out = formats.to_yaml(records)
        elif output == "sarif":
            out = formats.to_sarif(records)
        elif output == "junit":
            out = formats.to_junit(suites)
        else:
            raise ValueError(output)
    except GuardError as e:
        if raise_errors:
            raise
        return "", -1, "".join(stderr) + "Error occurred %s" % e.display()
    return out, exit_code, "".join(stderr)


# ---------------------------------------------------------------------------
# verbose EventRecord tree: serde's derived Serialize of EventRecord / RecordType
# (rules/mod.rs:165-355; externally tagged enums, struct fields in declaration order)
# ---------------------------------------------------------------------------
_QR_TAG = {"R": "Resolved", "L": "Literal", "U": "UnResolved"}


def _qr_json(q):
    if q is None:
        return None
    k, v = q
    return OMap([(_QR_TAG[k], _ur_json(v) if k == "U" else _pav_json(v))])


def _block_check(alo, status):
    return OMap([("at_least_one_matches", alo), ("status", status), ("message", None)])


def _clause_check_json(cc):
    k = cc[0]
    if k == "Success":
        return "Success"
    m = cc[1]
    if k == "Comparison":
        return OMap([(k, OMap([("comparison", list(m["comparison"])), ("from", _qr_json(m["from"])),
                               ("to", _qr_json(m["to"])), ("message", m["message"]),
                               ("custom_message", m["custom_message"]), ("status", m["status"])]))])
    if k == "InComparison":
        return OMap([(k, OMap([("comparison", list(m["comparison"])), ("from", _qr_json(m["from"])),
                               ("to", [_qr_json(t) for t in m["to"]]), ("message", m["message"]),
                               ("custom_message", m["custom_message"]), ("status", m["status"])]))])
    if k == "Unary":
        return OMap([(k, OMap([("value", OMap([("from", _qr_json(m["from"])), ("message", m["message"]),
                                                ("custom_message", m["custom_message"]), ("status", E.FAIL)])),
                               ("comparison", list(m["comparison"]))]))])
    if k == "NoValueForEmptyCheck":
        return OMap([(k, m)])
    if k == "DependentRule":
        return OMap([(k, OMap([("rule", m["rule"]), ("message", None), ("custom_message", m["custom_message"]),
                               ("status", E.FAIL)]))])
    # MissingBlockValue(ValueCheck)
    return OMap([(k, OMap([("from", _qr_json(m["from"])), ("message", m["message"]),
                           ("custom_message", m["custom_message"]), ("status", E.FAIL)]))])


def _container_json(c):
    k = c[0]
    if k in ("FileCheck", "RuleCheck"):
        return OMap([(k, OMap([("name", c[1]), ("status", c[2]), ("message", c[3] if len(c) > 3 else None)]))])
    if k in ("RuleCondition", "TypeCondition", "TypeBlock", "Filter", "WhenCondition"):
        return OMap([(k, c[1])])
    if k == "TypeCheck":
        return OMap([(k, OMap([("type_name", c[2]), ("block", _block_check(False, c[1]))]))])
    if k == "WhenCheck":
        return OMap([(k, _block_check(False, c[1]))])
    if k == "Disjunction":
        return OMap([(k, _block_check(True, c[1]))])
    if k in ("BlockGuardCheck", "GuardClauseBlockCheck"):
        return OMap([(k, _block_check(c[2], c[1]))])
    return OMap([(k, _clause_check_json(c[1]))])


# ---------------------------------------------------------------------------
# verbose EventRecord tree as text: Display of EventRecord / RecordType / ClauseCheck (display.rs:
# 128-328) drawn by pprint_tree (commands/validate.rs:666-687) -- `cfn-guard test --verbose`
# (reporters/test/generic.rs:116-118) and `validate --verbose`
# ---------------------------------------------------------------------------
_CMP_DISPLAY = {"Eq": "EQUALS", "In": "IN", "Gt": "GREATER THAN", "Lt": "LESS THAN", "Ge": "GREATER THAN EQUALS",
                "Le": "LESS THAN EQUALS", "Exists": "EXISTS", "Empty": "EMPTY", "IsString": "IS STRING",
                "IsBool": "IS BOOL", "IsInt": "IS INT", "IsList": "IS LIST", "IsMap": "IS MAP", "IsNull": "IS NULL",
                "IsFloat": "IS FLOAT"}


def _cmp_text(c):
    """display_comparison (display.rs:9-11): format!("{} {}", if not {"not"} else {""}, cmp)"""
    op, neg = c
    return "%s %s" % ("not" if neg else "", _CMP_DISPLAY[op])


def _qr_text(q):
    """QueryResult Display (display.rs:109-126)"""
    k, v = q
    if k == "L":
        return "literal, %s" % P.display(v)
    if k == "R":
        return "(resolved, %s)" % P.display(v)
    return "(unresolved, %s)" % P.display(v.traversed_to)


def _slice_text(items):
    """SliceDisplay (exprs.rs:286-303): items joined by "." with ".[" -> "[" """
    return ".".join(items).replace(".[", "[")


def _container_text(c):
    k = c[0]
    if k == "FileCheck":
        return "File(%s, Status=%s)" % (c[1], c[2])
    if k == "RuleCheck":
        return "Rule(%s, Status=%s)" % (c[1], c[2])
    if k == "RuleCondition":
        return "Rule/When(Status=%s)" % c[1]
    if k == "TypeCheck":
        return "Type(%s, Status=%s)" % (c[2], c[1])
    if k == "TypeCondition":
        return "TypeBlock/When Status=%s)" % c[1]
    if k == "TypeBlock":
        return "TypeBlock/Block Status=%s)" % c[1]
    if k == "Filter":
        return "Filter/ConjunctionsBlock(Status=%s)" % c[1]
    if k == "WhenCheck":
        return "WhenConditionalBlock(Status = %s)" % c[1]
    if k == "WhenCondition":
        return "WhenCondition(Status = %s)" % c[1]
    if k == "Disjunction":
        return "Disjunction(Status = %s)" % c[1]
    if k == "BlockGuardCheck":
        return "GuardValueBlockCheck(Status = %s)" % c[1]
    if k == "GuardClauseBlockCheck":
        return "GuardClauseBlock(Status = %s)" % c[1]
    cc = c[1]
    ck = cc[0]
    if ck == "Success":
        return "GuardClauseValueCheck(Status=PASS)"
    m = cc[1]
    if ck == "NoValueForEmptyCheck":
        return "GuardClause(Status=FAIL, Empty, %s)" % (m or "")
    if ck == "MissingBlockValue":
        f = m["from"]
        tt = P.display_path_only(f[1].traversed_to) if f[0] == "U" else ""
        return "GuardBlockValueMissing(Status=FAIL, Reason=%s, %s)" % (m["message"] or "", tt)
    if ck == "DependentRule":
        return "GuardClauseDependentRule(Rule=%s, Status=FAIL)" % m["rule"]
    if ck == "Unary":
        return "GuardClauseUnaryCheck(Status=FAIL, Comparison=%s, Value-At=%s)" % (_cmp_text(m["comparison"]), _qr_text(m["from"]))
    if ck == "Comparison":
        return "GuardClauseBinaryCheck(Status=%s, Comparison=%s, from=%s, to=%s)" % (
            m["status"], _cmp_text(m["comparison"]), _qr_text(m["from"]), _qr_text(m["to"]) if m["to"] is not None else "")
    return "GuardClauseInBinaryCheck(Status=%s, Comparison=%s, from=%s, to=%s)" % (
        m["status"], _cmp_text(m["comparison"]), _qr_text(m["from"]), _slice_text([_qr_text(t) for t in m["to"]]))


def event_text(ev):
    """print_verbose_tree: pprint_tree(root, "", true) -- one line per record,
    prefix + ("`- " | "|- ") + "{container}[Context={context}]" """
    out = []

    def walk(e, prefix, last):
        out.append("%s%s%s[Context=%s]\n" % (prefix, "`- " if last else "|- ", _container_text(e.container), e.context))
        child_prefix = prefix + ("   " if last else "|  ")
        for i, ch in enumerate(e.children):
            walk(ch, child_prefix, i == len(e.children) - 1)
    walk(ev, "", True)
    return "".join(out)


def event_json(ev):
    """EventRecord {context, container, children} (eval_context.rs:990-997)"""
    return OMap([("context", ev.context), ("container", _container_json(ev.container)),
                 ("children", [event_json(ch) for ch in ev.children])])


def run_checks(data_text, data_name, rules_text, rules_name, verbose=False):
    """guard-ffi ``run_checks`` (commands/helper.rs:25-87).
    Returns the pretty FileReport JSON (verbose: the pretty EventRecord tree of the evaluation,
    helper.rs:62-64) or raises GuardError."""
    from .loader import load_serde_json
    try:
        doc = load_serde_json(data_text)
    except GuardError:
        raise
    except Exception:
        raise GuardError("Unsupported", "serde_yaml fallback is outside the oracle's scope")
    rf = parse_rules(rules_text, rules_name)
    if rf is None:
        return ""
    if verbose:
        root = E.RootScope(rf, doc)
        E.eval_rules_file(rf, root, data_name)
        return to_json_pretty(event_json(root.recorder.final_event))
    st, rep = eval_file_report(rf, doc, data_name)
    return to_json_pretty(OMap([
        ("name", rep["name"]), ("metadata", OMap([])), ("status", rep["status"]),
        ("not_compliant", [_clause_json(c) for c in rep["not_compliant"]]),
        ("not_applicable", sorted(rep["not_applicable"], key=_rust_str_key)),
        ("compliant", sorted(rep["compliant"], key=_rust_str_key))]))
