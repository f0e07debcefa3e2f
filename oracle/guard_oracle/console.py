"""Console (non-structured) `cfn-guard validate` reporters (TEST INFRASTRUCTURE ONLY -- the parity oracle).

Restates, over the oracle's EventRecord trees:

* ``evaluate_rule`` / ``evaluate_against_data_input`` / ``print_verbose_tree``
  (``guard/src/commands/validate.rs:552-596, 666-758``) -- the per rules file x data file loop, exit
  codes, ``--verbose`` and ``--print-json``;
* the reporter chain ``SummaryTable -> CfnAware -> TfAware -> GenericSummary``
  (``reporters/validate/summary_table.rs:152-239``, ``cfn.rs:64-411``, ``tf.rs:43-301``,
  ``generic_summary.rs:116-307``) and its helpers in ``reporters/validate/common.rs``
  (``find_failing_clauses`` 134-160, ``extract_name_info_from_record`` 162-331, ``report_from_events``
  333-382, ``print_name_info`` 497-634, ``populate_hierarchy_path_trees`` 700-761,
  ``emit_messages`` / ``emit_retrieval_error`` / ``pprint_clauses`` 763-1198);
* ``utils::ReadCursor`` (``guard/src/utils/mod.rs:7-65``) for the CFN reporter's code snippets,
  including its line-number bookkeeping when it seeks backwards;
* ``Traversal`` (``rules/path_value/traversal.rs``) as a path -> value map.

The reference iterates Rust ``HashMap`` / ``HashSet`` values in three places (the CFN / TF
reporters' resources, the generic reporter's failed rules, its passed / skipped rule sets); their
order is ``RandomState``-random per process.  This restatement uses first-insertion order there (the
MI355X build does the same); outputs with one entry in each are the reference's bytes.  Colours are
off (the ``colored`` crate's behaviour when stdout is not a terminal, as in the reference's tests).
"""
import re

from . import evaluator as E
from . import pv as P
from .errors import GuardError
from .loader import load_document
from .parser import parse_rules
from .report import (OMap, simplified_json_from_root, file_report_json, to_json_pretty, event_text, event_json,
                     _json_str)

PASS_F, FAIL_F, SKIP_F = 1, 2, 4


class Panic(GuardError):
    """a Rust panic (unreachable!() / todo!() / unwrap on None) -- the CLI aborts"""

    def __init__(self, msg):
        GuardError.__init__(self, "Panic", msg)


class _Internal(Exception):
    """InternalError(UnresolvedKeyForReporter): the CFN reporter hands over to the next one"""


def summary_flags(values):
    """validate.rs:254-268: fold of --show-summary values; `none` resets to empty"""
    st = 0
    for v in values:
        if v == "none":
            st = 0
            continue
        st |= {"pass": PASS_F, "fail": FAIL_F, "skip": SKIP_F, "all": PASS_F | FAIL_F | SKIP_F}[v]
    return st


def _status_str(s):
    return {E.PASS: "PASS", E.FAIL: "FAIL", E.SKIP: "SKIP"}[s]


def get_rule_name(rules_file, name):
    """parser.rs:1828-1835"""
    pre = rules_file + "/"
    return name[len(pre):] if name.startswith(pre) else name


def _blen(s):
    return len(s.encode("utf-8", "surrogatepass"))


def _pad(s, width):
    # `{:<width$}`: pads to `width` chars (Rust counts chars)
    return s + " " * max(0, width - len(s))


# ------------------------------------------------------------------------- summary table ----------
def summary_table(out, status, root, rules_file, data_file, flags):
    """SummaryTable::report_eval (summary_table.rs:152-239)"""
    passed, skipped, failed = {}, {}, {}
    longest = 0
    for ch in root.children:
        c = ch.container
        if c is not None and c[0] == "RuleCheck":
            name, st = c[1], c[2]
            {E.PASS: passed, E.FAIL: failed, E.SKIP: skipped}[st][name] = st
            longest = max(longest, _blen(get_rule_name(rules_file, name)))
    skipped = {k: v for k, v in skipped.items() if k not in passed and k not in failed}
    wrote = False

    def header():
        out.append("%s Status = %s\n" % (data_file, _status_str(status)))

    def section(title, rules):
        for name, st in rules.items():
            out.append("%s/%s%s\n" % (rules_file, _pad(get_rule_name(rules_file, name), longest + 4), _status_str(st)))

    if flags & SKIP_F and skipped:
        header()
        wrote = True
        out.append("SKIP rules\n")
        section("SKIP", skipped)
    if flags & PASS_F and passed:
        if not wrote:
            wrote = True
            header()
        out.append("PASS rules\n")
        section("PASS", passed)
    if flags & FAIL_F and failed:
        if not wrote:
            wrote = True
            header()
        out.append("FAILED rules\n")
        section("FAIL", failed)
    if wrote:
        out.append("---\n")


# ------------------------------------------------------------------------- common helpers --------
def traversal(doc):
    """Traversal::from (traversal.rs:171-187): every value by its path (a later value with the same
    path replaces an earlier one, BTreeMap::insert), and "/" for the root"""
    nodes = {}

    def walk(v):
        nodes[v.path] = v
        if v.kind == P.MAP:
            for e in v.val.values.values():
                walk(e)
        elif v.kind == P.LIST:
            for e in v.val:
                walk(e)
    walk(doc)
    nodes["/"] = doc
    return nodes


def _skey(s):
    return s.encode("utf-8", "surrogatepass")


def cmp_str(cmp):
    """eval_context.rs:1847-1962"""
    op, neg = cmp
    unary = {"Exists": ("NOT EXISTS", "EXISTS"), "Empty": ("NOT EMPTY", "EMPTY"), "IsList": ("NOT LIST", "IS LIST"),
             "IsMap": ("NOT STRUCT", "IS STRUCT"), "IsString": ("NOT STRING", "IS STRING"),
             "IsFloat": ("NOT FLOAT", "IS FLOAT"), "IsNull": ("NOT NULL", "IS NULL"), "IsBool": ("NOT BOOL", "IS BOOl"),
             "IsInt": ("NOT INT", "IS INT"), "Eq": ("NOT EQUAL", "EQUAL"), "Le": ("NOT LESS THAN EQUAL", "LESS THAN EQUAL"),
             "Lt": ("NOT LESS THAN", "LESS THAN"), "Ge": ("NOT GREATER THAN EQUAL", "GREATER THAN EQUAL"),
             "Gt": ("NOT GREATER THAN", "GREATER THAN"), "In": ("NOT IN", "IN")}
    a, b = unary[op]
    return a if neg else b


class ReadCursor:
    """utils/mod.rs:7-65, line-for-line (including the numbering it records when seek_line runs
    forward from a position it reached by seeking backwards)"""

    def __init__(self, text):
        lines = text.split("\n")
        if lines and lines[-1] == "":
            lines.pop()
        self.src = iter([l[:-1] if l.endswith("\r") else l for l in lines])
        self.line_num = 0
        self.prev = []

    def next(self):
        if self.line_num < len(self.prev):
            self.line_num += 1
            return self.prev[self.line_num - 1]
        line = next(self.src, None)
        if line is None:
            return None
        self.line_num += 1
        self.prev.append((self.line_num, line))
        return self.prev[self.line_num - 1]

    def seek_line(self, line):
        if len(self.prev) > line:
            self.line_num = line
            return self.prev[self.line_num - 1]
        while True:
            l = next(self.src, None)
            if l is None:
                return None
            self.line_num += 1
            self.prev.append((self.line_num, l))
            if self.line_num == line:
                return self.prev[self.line_num - 1]


def _items(o):
    return dict(o.items)


def _clause_key(clause, parent):
    """ClauseReport::key (eval_context.rs:1799-1806); Block / Or / C use the clause's address"""
    kind, body = clause
    if kind == "Rule":
        return "%s/%s" % (parent, _items(body)["name"])
    tag = {"Block": "B", "Disjunctions": "Or", "Clause": "C"}[kind]
    return "%s/%s[%#x]" % (parent, tag, id(clause))


def _check_of(clause):
    """(kind, check-name, check-body) of a Clause report"""
    sub, body = clause[1]
    (cname, cbody), = _items(body)["check"].items
    return sub, cname, cbody


def _value_from(clause):
    kind, body = clause
    if kind == "Block":
        u = _items(body)["unresolved"]
        return None if u is None else u.pv
    if kind != "Clause":
        return None
    sub, cname, cbody = _check_of(clause)
    if cname == "UnResolvedContext":
        return None
    d = _items(cbody)
    if cname == "UnResolved":
        return d["value"].pv
    if cname == "Resolved":
        return d["value"].pv if sub == "Unary" else d["from"].pv
    return d["from"].pv   # InResolved


def _value_to(clause):
    if clause[0] != "Clause":
        return None
    sub, cname, cbody = _check_of(clause)
    if sub == "Binary" and cname == "Resolved":
        return _items(cbody)["to"].pv
    return None


def populate(clause, parent, path_tree):
    """populate_hierarchy_path_trees (common.rs:700-761): value path -> [(node path, clause)]"""
    kind, body = clause
    path = _clause_key(clause, parent)
    if kind in ("Clause", "Block"):
        for v in (_value_from(clause), _value_to(clause)):
            if v is not None:
                path_tree.setdefault(v.path, []).append((path, clause))
    else:
        for ch in _items(body)["checks"]:
            populate(ch, path, path_tree)


# char::is_whitespace (str::trim) -- Python's str.strip() would also take U+001C..U+001F
_RUST_WS = "\t\n\x0b\x0c\r \x85\xa0\u1680\u2000\u2001\u2002\u2003\u2004\u2005\u2006\u2007\u2008\u2009\u200a" \
           "\u2028\u2029\u202f\u205f\u3000"


def emit_messages(out, prefix, message, error, width):
    """common.rs:763-824"""
    if message:
        if ";" in message:
            parts = message.split(";")
        elif "\n" in message:
            parts = message.split("\n")
        else:
            parts = [message]
        parts = [p.strip(_RUST_WS) for p in parts]
        parts = [p for p in parts if p]
        if not parts:
            raise Panic("index out of bounds: the len is 0 but the index is 0")
        if len(parts) > 1:
            out.append("%s%s {\n" % (prefix, _pad("Message", width)))
            for p in parts:
                out.append("%s  %s\n" % (prefix, p))
            out.append("%s}\n" % prefix)
        else:
            out.append("%s%s = %s\n" % (prefix, _pad("Message", width), parts[0]))
    if error:
        out.append("%s%s = %s\n" % (prefix, _pad("Error", width), error))


def _msgs(body):
    m = _items(_items(body)["messages"])
    return m["custom_message"] or "", m["error_message"] or ""


def emit_retrieval_error(out, prefix, vur, clause, context, message, ew):
    """common.rs:826-872"""
    out.append("%sCheck = %s {\n" % (prefix, context))
    check_end = prefix + "}"
    prefix = prefix + "  "
    emit_messages(out, prefix, message, "", 0)
    out.append("%sRequiredPropertyError {\n" % prefix)
    rpe_end = prefix + "}"
    prefix = prefix + "  "
    ur = vur.ur
    out.append("%sPropertyPath = %s\n" % (prefix, ur.traversed_to.path_display()))
    out.append("%sMissingProperty = %s\n" % (prefix, ur.remaining_query))
    if ur.reason:
        out.append("%sReason = %s\n" % (prefix, ur.reason))
    ew.missing_property_msg(out, clause, ur, prefix)
    out.append(rpe_end + "\n")
    out.append(check_end + "\n")


def pprint_clauses(out, clause, resource, prefix, ew):
    """common.rs:911-1198"""
    kind, body = clause
    d = _items(body) if kind != "Clause" else None
    if kind == "Rule":
        out.append("%sRule = %s {\n" % (prefix, d["name"]))
        rule_end = prefix + "}"
        prefix = prefix + "  "
        custom, error = _msgs(body)
        emit_messages(out, prefix, custom, error, 0)
        out.append("%sALL {\n" % prefix)
        all_end = prefix + "}"
        for ch in d["checks"]:
            pprint_clauses(out, ch, resource, prefix + "  ", ew)
        out.append(all_end + "\n")
        out.append(rule_end + "\n")
        return
    if kind == "Disjunctions":
        out.append("%sANY {\n" % prefix)
        for ch in d["checks"]:
            pprint_clauses(out, ch, resource, prefix + "  ", ew)
        out.append(prefix + "}\n")
        return
    if id(clause) not in resource["clauses"]:
        return
    if kind == "Block":
        out.append("%sCheck = %s {\n" % (prefix, d["context"]))
        check_end = prefix + "}"
        prefix = prefix + "  "
        out.append("%sRequiredPropertyError {\n" % prefix)
        mpv_end = prefix + "}"
        prefix = prefix + "  "
        u = d["unresolved"]
        traversed, query = ("", "") if u is None else (u.ur.traversed_to.path, u.ur.remaining_query)
        if traversed:
            width = len("MissingProperty") + 4
            out.append("%s%s= %s\n%s%s= %s\n" % (prefix, _pad("PropertyPath", width), traversed,
                                                 prefix, _pad("MissingProperty", width), query))
        else:
            width = len("Message") + 4
        post = []
        width = max(width, ew.missing_property_msg(post, clause, None if u is None else u.ur, prefix))
        custom, error = _msgs(body)
        emit_messages(out, prefix, custom, error, width)
        out.append("".join(post) + "\n")
        out.append(mpv_end + "\n")
        out.append(check_end + "\n")
        return
    sub, cname, cbody = _check_of(clause)
    inner = _items(clause[1][1])
    custom, error = _msgs(clause[1][1])
    if cname == "UnResolved":
        emit_retrieval_error(out, prefix, _items(cbody)["value"], clause, inner["context"], custom, ew)
        return
    if cname == "UnResolvedContext":
        return
    out.append("%sCheck = %s {\n" % (prefix, inner["context"]))
    check_end = prefix + "}"
    prefix = prefix + "  "
    out.append("%sComparisonError {\n" % prefix)
    ce_end = prefix + "}"
    prefix = prefix + "  "
    post = []
    cb = _items(cbody)
    if sub == "Unary":
        width = ew.unary_error_msg(post, clause, cb, prefix)
    elif cname == "Resolved":
        width = ew.binary_error_msg(post, clause, cb, prefix)
    else:
        width = ew.binary_error_in_msg(post, clause, cb, prefix)
    emit_messages(out, prefix, custom, error, width)
    if cname == "InResolved":
        out.append(ce_end + "\n")
        out.append("".join(post) + "\n")
    else:
        out.append("".join(post) + "\n")
        out.append(ce_end + "\n")
    out.append(check_end + "\n")


class _CfnErr:
    """cfn.rs:255-411 ErrWriter: value lines plus the template's code around the value's line"""

    def __init__(self, cursor):
        self.cursor = cursor

    def emit_code(self, out, line, prefix):
        out.append("%sCode:\n" % prefix)
        np = prefix + "  "
        target = line - 2 if line >= 2 else (1 << 64) + line - 2   # usize arithmetic wraps (release build)
        hit = self.cursor.seek_line(max(1, target))
        if hit is not None:
            out.append("%s%5d.%s\n" % (np, hit[0], hit[1]))
        context = 5
        while True:
            nx = self.cursor.next()
            if nx is None:
                break
            out.append("%s%5d.%s\n" % (np, nx[0], nx[1]))
            context -= 1
            if context <= 0:
                break

    def missing_property_msg(self, out, clause, ur, prefix):
        if ur is not None:
            self.emit_code(out, ur.traversed_to.line, prefix)
        return 0

    def binary_error_msg(self, out, clause, cb, prefix):
        w = len("PropertyPath") + 4
        frm, to = cb["from"].pv, cb["to"].pv
        out.append("%s%s= %s\n%s%s= %s\n%s%s= %s\n%s%s= %s\n" % (
            prefix, _pad("PropertyPath", w), frm.path_display(), prefix, _pad("Operator", w), cmp_str(cb["comparison"]),
            prefix, _pad("Value", w), P.value_only(frm), prefix, _pad("ComparedWith", w), P.value_only(to)))
        self.emit_code(out, frm.line, prefix)
        return w

    def binary_error_in_msg(self, out, clause, cb, prefix):
        frm = cb["from"].pv
        to = [t.pv for t in cb["to"]]
        cut_off = max(len(to), 5)
        collected = []
        for idx, each in enumerate(to):
            collected.append(P.value_only(each))
            if idx >= cut_off:
                break
        collected = "[" + ", ".join(collected) + "]"
        w = len("PropertyPath") + 4
        out.append("%s%s= %s\n%s%s= %s\n%s%s= %s\n%s%s= %s\n" % (
            prefix, _pad("PropertyPath", w), frm.path_display(), prefix, _pad("Operator", w), cmp_str(cb["comparison"]),
            prefix, _pad("Value", w), P.value_only(frm), prefix, _pad("ComparedWith", w), collected))
        self.emit_code(out, frm.line, prefix)
        return w

    def unary_error_msg(self, out, clause, cb, prefix):
        w = len("PropertyPath") + 4
        v = cb["value"].pv
        out.append("%s%s= %s\n%s%s= %s\n" % (prefix, _pad("PropertyPath", w), v.path_display(),
                                             prefix, _pad("Operator", w), cmp_str(cb["comparison"])))
        self.emit_code(out, v.line, prefix)
        return w


class _TfErr:
    """tf.rs:205-289 ErrWriter (no code snippets)"""

    def missing_property_msg(self, out, clause, ur, prefix):
        return 0

    def binary_error_msg(self, out, clause, cb, prefix):
        w = len("PropertyPath") + 4
        frm, to = cb["from"].pv, cb["to"].pv
        based = frm.path if frm.path.startswith("/resource_changes") else to.path
        i = based.find("change/after/")
        prop = "" if i < 0 else based[i:]
        prop = prop[len("change/after/"):].replace("/", ".")
        out.append("%s%s= %s\n%s%s= %s\n%s%s= %s\n%s%s= %s\n" % (
            prefix, _pad("PropertyPath", w), prop, prefix, _pad("Operator", w), cmp_str(cb["comparison"]),
            prefix, _pad("Value", w), P.value_only(frm), prefix, _pad("ComparedWith", w), P.value_only(to)))
        return w

    def binary_error_in_msg(self, out, clause, cb, prefix):
        raise Panic("not yet implemented")

    def unary_error_msg(self, out, clause, cb, prefix):
        w = len("PropertyPath") + 4
        based = cb["value"].pv.path
        i = based.find("changes/after/")
        prop = ("" if i < 0 else based[i:]).replace("/", ".")
        out.append("%s%s= %s\n%s%s= %s\n" % (prefix, _pad("PropertyPath", w), prop,
                                             prefix, _pad("Operator", w), cmp_str(cb["comparison"])))
        return w


def _print_resources(out, data_file, rules_file, not_compliant, by_res, ew):
    out.append("Evaluating data %s against rules %s\n" % (data_file, rules_file))
    out.append("Number of non-compliant resources %d\n" % len(by_res))
    for res in by_res.values():
        out.append("Resource = %s {\n" % res["name"])
        prefix = "  "
        out.append("%s%s= %s\n" % (prefix, _pad("Type", 10), res["type"]))
        if res["cdk"]:
            out.append("%s%s= %s\n" % (prefix, _pad("CDK-Path", 10), res["cdk"]))
        for rule in not_compliant:
            if rule[0] != "Rule":
                raise Panic("internal error: entered unreachable code")
            rn = "/" + _items(rule[1])["name"]
            if any(p.startswith(rn) for p in res["paths"]):
                pprint_clauses(out, rule, res, prefix, ew)
        out.append("}\n")


CFN_RESOURCES = re.compile(r"^/Resources/([^/]+)(/?P<rest>.*$)?")


def _get_resource_name(key, count, matches):
    """cfn.rs:427-444"""
    c = "\x0c"
    ph = key.replace("/", c, matches - count)
    ph = ph.replace(c, "/", 2)
    m = CFN_RESOURCES.match(ph)
    if not m:
        raise Panic("internal error: entered unreachable code")
    return m.group(1).replace(c, "/")


def _resource_aggr(paths, name, by_res, nodes):
    """cfn.rs:446-503"""
    path = "/Resources/" + name
    res = paths.get(path)
    if res is None:
        return False
    t = paths.get(res.path + "/Type")
    if t is None:
        return False
    if t.kind != P.STRING:
        raise Panic("internal error: entered unreachable code")
    cdk = paths.get(res.path + "/Metadata/aws:cdk:path")
    if cdk is not None and cdk.kind != P.STRING:
        raise Panic("internal error: entered unreachable code")
    agg = by_res.get(name)
    if agg is None:
        agg = by_res[name] = {"name": name, "type": t.val, "cdk": None if cdk is None else cdk.val,
                              "clauses": set(), "paths": set()}
    for npath, clause in nodes:
        agg["clauses"].add(id(clause))
        agg["paths"].add(npath)
    return True


def cfn_single_line(out, data_file, text, rules_file, paths, fr):
    """cfn.rs:143-425"""
    nc = fr["not_compliant"]
    if not nc:
        return
    tree = {}
    for r in nc:
        populate(r, "", tree)
    by_res = {}
    for key in sorted((k for k in tree if _skey(k) >= _skey("/Resources")), key=_skey):
        nodes = tree[key]
        matches = key.count("/")
        if matches > 2:
            count = 1
            while True:
                if matches - count == 0:
                    raise Panic("internal error: entered unreachable code")
                if _resource_aggr(paths, _get_resource_name(key, count, matches), by_res, nodes):
                    break
                count += 1
        else:
            m = CFN_RESOURCES.match(key)
            if not m:
                raise _Internal()
            if not _resource_aggr(paths, m.group(1), by_res, nodes):
                raise Panic("internal error: entered unreachable code")
    _print_resources(out, data_file, rules_file, nc, by_res, _CfnErr(ReadCursor(text)))


RESOURCE_CHANGE = re.compile(r"/resource_changes/([^/]+)/change/after/(.*)?")


def tf_single_line(out, data_file, rules_file, paths, fr):
    """tf.rs:101-301"""
    nc = fr["not_compliant"]
    if not nc:
        return
    tree = {}
    for r in nc:
        populate(r, "", tree)
    by_res = {}
    for key in sorted((k for k in tree if _skey(k) >= _skey("/resource_changes/")), key=_skey):
        m = RESOURCE_CHANGE.search(key)
        if not m:
            raise Panic("internal error: entered unreachable code")
        address = "/resource_changes/" + m.group(1)
        res = paths.get(address)
        if res is None:
            raise GuardError("RetrievalError", "Path %s did not yield value" % address)
        addr = paths.get(res.path + "/address")
        if addr is None:
            raise GuardError("RetrievalError", "Path %s/address did not yield value" % res.path)
        if addr.kind != P.STRING:
            raise Panic("internal error: entered unreachable code")
        dot = addr.val.find(".")
        if dot < 0:
            raise Panic("called `Option::unwrap()` on a `None` value")
        rtype, rname = addr.val[:dot], addr.val[dot + 1:]
        agg = by_res.get(rname)
        if agg is None:
            agg = by_res[rname] = {"name": rname, "type": rtype, "cdk": None, "clauses": set(), "paths": set()}
        for npath, clause in tree[key]:
            agg["clauses"].add(id(clause))
            agg["paths"].add(npath)
    _print_resources(out, data_file, rules_file, nc, by_res, _TfErr())


# ------------------------------------------------------------------------- generic reporter ------
def _json_compact(o):
    """serde_json::Value Display (compact; preserve_order maps)"""
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
    if isinstance(o, dict):
        return "{" + ",".join("%s:%s" % (_json_str(k), _json_compact(v)) for k, v in o.items()) + "}"
    if isinstance(o, list):
        return "[" + ",".join(_json_compact(v) for v in o) + "]"
    raise TypeError(type(o))


def find_failing_clauses(cur):
    """common.rs:134-160"""
    c = cur.container
    if c is not None:
        if c[0] == "Filter" or (c[0] == "ClauseValueCheck" and c[1][0] == "Success"):
            return []
        if c[0] == "ClauseValueCheck":
            return [cur]
        if c[0] == "RuleCheck" and c[3] is not None and c[2] == E.FAIL:
            return [cur]
    acc = []
    for ch in cur.children:
        acc.extend(find_failing_clauses(ch))
    return acc


def _qr_json_value(q):
    k, v = q
    return P.to_json_value(v.traversed_to if k == "U" else v)


def _info(rule, **kw):
    d = {"rule": rule, "path": "", "provided": None, "expected": None, "comparison": None, "message": "", "error": None}
    d.update(kw)
    return d


def extract_name_info(rule_name, ev):
    """common.rs:162-331"""
    c = ev.container
    if c[0] == "RuleCheck":
        return _info(c[1], message=c[3])
    k, m = c[1][0], (c[1][1] if len(c[1]) > 1 else None)
    if k == "DependentRule":
        return _info(rule_name, error=None, message=m["custom_message"] or "")
    if k == "MissingBlockValue":
        frm = m["from"]
        path = frm[1].traversed_to.path if frm[0] == "U" else ""
        return _info(rule_name, error=m.get("message"), message=m["custom_message"] or "", path=path)
    if k == "Unary":
        frm = m["from"]
        if frm[0] == "L":
            raise Panic("internal error: entered unreachable code")
        if frm[0] == "R":
            return _info(rule_name, comparison=tuple(m["comparison"]), error=m["message"],
                         message=m["custom_message"] or "", provided=P.to_json_value(frm[1]), path=frm[1].path)
        ur = frm[1]
        return _info(rule_name, comparison=tuple(m["comparison"]),
                     error=m["message"] if m["message"] is not None else (ur.reason or ""),
                     message=m["custom_message"] or "", provided=P.to_json_value(ur.traversed_to), path=ur.traversed_to.path)
    if k == "Comparison":
        frm = m["from"]
        if frm[0] == "L":
            raise Panic("internal error: entered unreachable code")
        if frm[0] == "R":
            to = m["to"]
            if to is not None and to[0] == "L":
                raise Panic("internal error: entered unreachable code")
            expected = None if to is None else _qr_json_value(to)
            return _info(rule_name, comparison=tuple(m["comparison"]), error=m["message"],
                         message=m["custom_message"] or "", provided=P.to_json_value(frm[1]), expected=expected,
                         path=frm[1].path)
        ur = frm[1]
        return _info(rule_name, comparison=tuple(m["comparison"]),
                     error=m["message"] if m["message"] is not None else (ur.reason or ""),
                     message=m["custom_message"] or "", provided=P.to_json_value(ur.traversed_to), path=ur.traversed_to.path)
    if k == "NoValueForEmptyCheck":
        return _info(rule_name, comparison=("Empty", False), message=m or "")
    if k == "InComparison":
        frm = m["from"]
        provided = P.to_json_value(frm[1]) if frm[0] == "R" else None
        to = []
        for t in m["to"]:
            to.append(P.to_json_value(t[1].traversed_to if t[0] == "U" else t[1]))
        return _info(rule_name, comparison=tuple(m["comparison"]), provided=provided, expected=to,
                     message=m["message"] or "")
    raise Panic("internal error: entered unreachable code")


_UNARY_OP_MSG = {"Exists": ("did not exist", "existed"), "Empty": ("was not empty", "was empty"),
                 "IsList": ("was not a list ", "was list"), "IsMap": ("was not a struct", "was struct"),
                 "IsString": ("was not a string ", "was string"), "IsBool": ("was not a bool", "was bool"),
                 "IsInt": ("was not an int", "was int"), "IsNull": ("was not null", "was null"),
                 "IsFloat": ("was not a float", "was float")}


def print_name_info(out, infos, data_file):
    """common.rs:497-634 with generic_summary.rs's message builders (185-254)"""
    for each in infos:
        if each["error"] is not None:
            out.append("Property traversed until [%s] in data [%s] is not compliant with [%s] due to retrieval error. "
                       "Error Message [%s]\n" % (each["path"], data_file, each["rule"], each["error"]))
            continue
        cmp = each["comparison"]
        if cmp is None:
            out.append("Parameterized Rule %s failed for %s. Reason %s\n" % (
                each["rule"], data_file, each["message"].replace("\n", "; ")))
            continue
        op, neg = cmp
        msg = each["message"].replace("\n", ";")
        provided = _json_compact(each["provided"])
        if op in _UNARY_OP_MSG:
            a, b = _UNARY_OP_MSG[op]
            out.append("Property [%s] in data [%s] is not compliant with [%s] because needed value at [%s] %s. "
                       "Error Message [%s]\n" % (each["path"], data_file, each["rule"], provided, b if neg else a, msg))
        else:
            out.append("Property [%s] in data [%s] is not compliant with [%s] because provided value [%s] %s %s [%s]. "
                       "Error Message [%s]\n" % (
                           each["path"], data_file, each["rule"], provided, "did" if neg else "did not",
                           "match expected value in" if op == "In" else "match expected value",
                           _json_compact(each["expected"]), msg))


def generic_single_line(out, root, rules_file, data_file, flags):
    """report_from_events (common.rs:333-382) + SingleLineSummary::report (generic_summary.rs:272-307)"""
    failed, passed, skipped = {}, {}, {}
    for rule in root.children:
        c = rule.container
        if c is None or c[0] != "RuleCheck":
            continue
        name, st = c[1], c[2]
        if st == E.FAIL:
            failed[name] = [extract_name_info(name, ev) for ev in find_failing_clauses(rule)]
        elif st == E.PASS:
            passed[name] = True
        else:
            skipped[name] = True
    if not flags:
        return
    if flags & FAIL_F:
        ok = bool(failed)
    elif flags & PASS_F:
        ok = bool(passed)
    else:
        ok = bool(skipped) and bool(flags & SKIP_F)
    if not ok:
        return
    out.append("Evaluation of rules %s against data %s\n" % (rules_file, data_file))
    if flags & FAIL_F:
        if failed:
            out.append("--\n")
        for infos in failed.values():
            print_name_info(out, infos, data_file)
    for bit, rules, what in ((PASS_F, passed, "compliant"), (SKIP_F, skipped, "not applicable")):
        if flags & bit:
            if rules:
                out.append("--\n")
            for r in rules:
                out.append("Rule [%s] is %s for template [%s]\n" % (r, what, data_file))
    out.append("--\n")


# ------------------------------------------------------------------------- the command -----------
def _file_report(root):
    return file_report_json(simplified_json_from_root(root))


def report_eval(out, status, root, rules_file, data_file, text, doc, output, flags):
    """SummaryTable (when flags) -> CfnAware -> TfAware -> GenericSummary"""
    if flags:
        summary_table(out, status, root, rules_file, data_file, flags)
    paths = traversal(doc)

    def structured():
        from . import formats
        fr = _file_report(root)
        out.append(to_json_pretty(fr) if output == "json" else formats.to_yaml(fr))

    if "/Resources" in paths:
        if output in ("json", "yaml"):
            return structured()
        part = []
        try:
            cfn_single_line(part, data_file, text, rules_file, paths, simplified_json_from_root(root))
            out.extend(part)
            return
        except _Internal:
            pass   # raised before anything is written: the next reporter runs
        except GuardError:
            out.extend(part)   # a panic mid-report: what was written stays written
            raise
    if "/resource_changes" in paths:
        if output in ("json", "yaml"):
            return structured()
        return tf_single_line(out, data_file, rules_file, paths, simplified_json_from_root(root))
    if output in ("json", "yaml"):
        return structured()
    generic_single_line(out, root, rules_file, data_file, flags)


def validate_console(rules, data, summary=("fail",), output="single-line-summary", verbose=False, print_json=False,
                     params=None):
    """``cfn-guard validate [-r ...]+ [-d ...]+ [-i ...]* [-o single-line-summary|json|yaml] [-S ...]
    [--verbose] [--print-json]`` over in-memory inputs (rules, data: lists of (name, text) in the CLI's
    walk order).  Returns (stdout, exit_code, stderr); an evaluation error ends the run with what was
    written so far and exit code -1 (main.rs), its Display in stderr."""
    flags = summary_flags(summary)
    out, err = [], []
    exit_code = 0
    try:
        docs = [(n, t, load_document(t, n)) for n, t in data]
        primary = None
        if params:
            from .pv import merge as pv_merge
            for n, t in params:
                pv = load_document(t, n)
                primary = pv if primary is None else pv_merge(primary, pv)
        for rname, rtext in rules:
            try:
                rf = parse_rules(rtext, rname)
            except GuardError as e:
                err.append("Parsing error handling rule file = %s, Error = %s\n---\n" % (rname, e.display()))
                exit_code = 5
                continue
            if rf is None:
                continue
            overall = E.PASS
            for dname, dtext, doc in docs:
                if primary is not None:   # validate.rs:719-722: `data.clone().merge(file)?` per file
                    doc = pv_merge(primary, doc)
                root = E.RootScope(rf, doc)
                st = E.eval_rules_file(rf, root, dname)
                rec = root.recorder.final_event
                report_eval(out, st, rec, rname, dname, dtext, doc, output, flags)
                if verbose:
                    out.append(event_text(rec))
                if print_json:
                    out.append(to_json_pretty(event_json(rec)) + "\n")
                if st == E.FAIL:
                    overall = E.FAIL
            if overall == E.FAIL:
                exit_code = 19
    except GuardError as e:
        return "".join(out), -1, "".join(err) + "Error occurred %s" % e.display()
    return "".join(out), exit_code, "".join(err)


__all__ = ["validate_console", "summary_flags", "ReadCursor", "OMap"]
