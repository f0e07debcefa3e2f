"""Document loader restatement (TEST INFRASTRUCTURE ONLY -- the parity oracle).

Restates ``guard/src/rules/libyaml/loader.rs:31-244`` (event-driven libyaml loader with
scalar typing, CFN short-form tags and (line, col) marks) and
``PathAwareValue::try_from((MarkedValue, Path))`` ``path_value.rs:414-478``.

The reference links unsafe-libyaml 0.2.11 (a mechanical Rust transpile of libyaml 0.2.5,
Cargo.lock).  PyYAML's bundled C libyaml here reports version 0.2.5, so its event stream and
marks are the same third-party algorithm; this module only consumes the events.

Also restates the guard-ffi / ``run_checks`` loader (``commands/helper.rs:30-42``:
serde_json first, then serde_yaml, every Location = L:0,C:0) in :func:`load_serde`.
"""
import json
import math
import re

from yaml._yaml import CParser

from .errors import GuardError
from .pv import rust_debug_str, PV, MapValue, STRING, INT, FLOAT, BOOL, NULL, LIST, MAP

SHORT_FORM_TO_LONG = {
    "Ref": "Ref", "GetAtt": "Fn::GetAtt", "Base64": "Fn::Base64", "Sub": "Fn::Sub",
    "GetAZs": "Fn::GetAZs", "ImportValue": "Fn::ImportValue", "Condition": "Condition",
    "RefAll": "Fn::RefAll", "Select": "Fn::Select", "Split": "Fn::Split", "Join": "Fn::Join",
    "FindInMap": "Fn::FindInMap", "And": "Fn::And", "Equals": "Fn::Equals",
    "Contains": "Fn::Contains", "EachMemberIn": "Fn::EachMemberIn",
    "EachMemberEquals": "Fn::EachMemberEquals", "ValueOf": "Fn::ValueOf", "If": "Fn::If",
    "Not": "Fn::Not", "Or": "Fn::Or",
}
SINGLE_VALUE_FUNC_REF = {"Ref", "Base64", "Sub", "GetAZs", "ImportValue", "GetAtt", "Condition", "RefAll"}
SEQUENCE_VALUE_FUNC_REF = {"GetAtt", "Sub", "Select", "Split", "Join", "FindInMap", "And", "Equals",
                           "Contains", "EachMemberIn", "EachMemberEquals", "ValueOf", "If", "Not", "Or"}
TYPE_REF_PREFIX = "tag:yaml.org,2002:"

_I64_RE = re.compile(r"^[+-]?[0-9]+$")
_F64_RE = re.compile(r"^[+-]?(?:[0-9]+\.?[0-9]*(?:[eE][+-]?[0-9]+)?|\.[0-9]+(?:[eE][+-]?[0-9]+)?)$")
_F64_SPECIAL = re.compile(r"^[+-]?(?:inf|infinity|nan)$", re.IGNORECASE)

I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


def rust_parse_i64(s):
    """``str::parse::<i64>``"""
    if not _I64_RE.match(s):
        return None
    v = int(s)
    if v < I64_MIN or v > I64_MAX:
        return None
    return v


def rust_parse_f64(s):
    """``str::parse::<f64>``"""
    if _F64_RE.match(s):
        return float(s)
    if _F64_SPECIAL.match(s):
        neg = s.startswith("-")
        body = s.lstrip("+-").lower()
        if body == "nan":
            return math.nan
        return -math.inf if neg else math.inf
    return None


class _M:
    """MarkedValue (values.rs:403-442)."""
    __slots__ = ("kind", "val", "line", "col")

    def __init__(self, kind, val, line, col):
        self.kind, self.val, self.line, self.col = kind, val, line, col


BAD = "BadValue"


def _split_tag(tag):
    handle = ""
    for ch in tag:
        if ch == "!":
            handle += ch
        else:
            break
    return handle, tag[len(handle):]


def _scalar(ev):
    line, col = ev.start_mark.line, ev.start_mark.column
    val = ev.value
    tag = ev.tag
    if tag is not None:
        handle, suffix = _split_tag(tag)
        if handle == "!":
            if suffix in SINGLE_VALUE_FUNC_REF:
                return _M(MAP, [((SHORT_FORM_TO_LONG[suffix], line, col), _M(STRING, val, line, col))], line, col)
            return _M(STRING, val, line, col)
        if suffix.startswith(TYPE_REF_PREFIX):
            t = suffix
            if t == "tag:yaml.org,2002:bool":
                if val == "true":
                    return _M(BOOL, True, line, col)
                if val == "false":
                    return _M(BOOL, False, line, col)
                return _M(STRING, val, line, col)
            if t == "tag:yaml.org,2002:int":
                i = rust_parse_i64(val)
                return _M(INT, i, line, col) if i is not None else _M(BAD, val, line, col)
            if t == "tag:yaml.org,2002:float":
                f = rust_parse_f64(val)
                return _M(FLOAT, f, line, col) if f is not None else _M(BAD, val, line, col)
            if t == "tag:yaml.org,2002:null":
                return _M(NULL, None, line, col)
            return _M(STRING, val, line, col)
        return _M(STRING, val, line, col)
    if ev.style != "":
        return _M(STRING, val, line, col)
    i = rust_parse_i64(val)
    if i is not None:
        return _M(INT, i, line, col)
    f = rust_parse_f64(val)
    if f is not None:
        return _M(FLOAT, f, line, col)
    if val in ("true", "yes", "on", "y"):
        return _M(BOOL, True, line, col)
    if val in ("false", "no", "off", "n"):
        return _M(BOOL, False, line, col)
    if val.lower() in ("~", "null"):
        return _M(NULL, None, line, col)
    return _M(STRING, val, line, col)


def load_marked(content: str):
    """Loader::load -- returns the first document as a MarkedValue tree."""
    try:
        parser = CParser(content)
    except Exception as e:  # pragma: no cover
        raise GuardError("ParseError", "error parsing file")
    stack = []
    last_container = []
    func_support = []  # (stack index, (fn_name, line, col))
    while True:
        try:
            ev = parser.get_event()
        except Exception:
            raise GuardError("ParseError", "error parsing file")
        if ev is None:
            raise GuardError("ParseError", "error parsing file")
        name = type(ev).__name__
        if name in ("StreamStartEvent", "DocumentStartEvent"):
            continue
        if name == "StreamEndEvent":
            # the reference would keep polling libyaml after STREAM-END and hit
            # unimplemented!() (a panic); surface it as an explicit error here
            raise GuardError("ParseError", "error parsing file")
        if name == "DocumentEndEvent":
            return stack.pop()
        if name == "MappingStartEvent":
            stack.append(_M(MAP, [], ev.start_mark.line, ev.start_mark.column))
            last_container.append(len(stack) - 1)
        elif name == "MappingEndEvent":
            idx = last_container.pop()
            kvs = stack[idx + 1:]
            del stack[idx + 1:]
            m = stack[-1]
            for j in range(0, len(kvs), 2):
                k, v = kvs[j], kvs[j + 1]
                if k.kind != STRING:
                    raise GuardError("InternalError",
                                     "non string type detected for key in a map at L:%d,C:%d, "
                                     "cfn-guard only supports keys that are string types" % (k.line, k.col))
                _map_insert(m.val, (k.val, k.line, k.col), v)
        elif name == "SequenceStartEvent":
            line, col = ev.start_mark.line, ev.start_mark.column
            if ev.tag is not None:
                handle, suffix = _split_tag(ev.tag)
                if handle == "!" and suffix in SEQUENCE_VALUE_FUNC_REF:
                    fn = SHORT_FORM_TO_LONG[suffix]
                    stack.append(_M(MAP, [((fn, line, col), _M(NULL, None, line, col))], line, col))
                    func_support.append((len(stack) - 1, (fn, line, col)))
            stack.append(_M(LIST, [], line, col))
            last_container.append(len(stack) - 1)
        elif name == "SequenceEndEvent":
            idx = last_container.pop()
            vals = stack[idx + 1:]
            del stack[idx + 1:]
            stack[-1].val.extend(vals)
            if func_support and func_support[-1][0] == idx - 1:
                _, key = func_support.pop()
                arr = stack.pop()
                m = stack[-1]
                if m.kind == MAP:
                    _map_insert(m.val, key, arr)
        elif name == "ScalarEvent":
            stack.append(_scalar(ev))
        elif name == "AliasEvent":
            raise GuardError("ParseError", "Guard does not currently support aliases")


def _map_insert(entries, key, value):
    # IndexMap<(String, Location), MarkedValue>::insert
    for i, (k, _) in enumerate(entries):
        if k == key:
            entries[i] = (k, value)
            return
    entries.append((key, value))


def marked_to_pv(m, path="", line=0, col=0):
    """PathAwareValue::try_from((MarkedValue, Path)) path_value.rs:414-478.
    (line, col) is the location already attached to ``path`` by the caller."""
    k = m.kind
    if k == LIST:
        out = []
        for i, e in enumerate(m.val):
            out.append(marked_to_pv(e, "%s/%d" % (path, i), e.line, e.col))
        return PV(LIST, path, line, col, out)
    if k == MAP:
        mv = MapValue()
        for (key, kl, kc), e in m.val:
            sub = path + "/" + key
            mv.values[key] = marked_to_pv(e, sub, e.line, e.col)
            mv.keys.append(PV(STRING, path, kl, kc, key))
        return PV(MAP, path, m.line, m.col, mv)
    if k == BAD:
        raise GuardError("ParseError", "Bad Value encountered parsing incoming file Value = %s, Loc = L:%d,C:%d"
                         % (m.val, m.line, m.col))
    return PV(k, path, m.line, m.col, m.val)


def load_document(content: str, name: str = "DATA"):
    """``build_data_file`` (commands/validate.rs:760-787) + root conversion."""
    if content.strip() == "":
        raise GuardError("ParseError", "Unable to parse a template from data file: %s is empty" % name)
    try:
        m = load_marked(content)
    except GuardError as e:
        if e.kind == "InternalError":
            raise GuardError("ParseError", e.display())
        raw = content.encode("utf-8")[:100]
        raise GuardError("ParseError", "Error encountered while parsing data file: %s, data beginning with \n%s\n ..."
                         % (name, raw.decode("utf-8", "replace")))
    return marked_to_pv(m, "", 0, 0)


# ---------------------------------------------------------------------------
# serde loader (guard-ffi run_checks): commands/helper.rs:30-42, values.rs:287-366
# ---------------------------------------------------------------------------
def _from_serde_json(v, path):
    if v is None:
        return PV(NULL, path, 0, 0)
    if isinstance(v, bool):
        return PV(BOOL, path, 0, 0, v)
    if isinstance(v, int):
        if v > I64_MAX:
            v = v - (1 << 64) if v < (1 << 64) else None
            if v is None:
                raise GuardError("JsonError", "number out of range")
        return PV(INT, path, 0, 0, v)
    if isinstance(v, float):
        return PV(FLOAT, path, 0, 0, v)
    if isinstance(v, str):
        return PV(STRING, path, 0, 0, v)
    if isinstance(v, list):
        return PV(LIST, path, 0, 0, [_from_serde_json(e, "%s/%d" % (path, i)) for i, e in enumerate(v)])
    mv = MapValue()
    for key in v:
        mv.keys.append(PV(STRING, path + "/" + key, 0, 0, key))
    for key, e in v.items():
        mv.values[key] = _from_serde_json(e, path + "/" + key)
    return PV(MAP, path, 0, 0, mv)


def _json_pairs(pairs):
    d = {}
    for k, v in pairs:
        d[k] = v  # serde_json(preserve_order): last value, first position
    return d


def load_serde_json(content: str):
    v = json.loads(content, object_pairs_hook=_json_pairs,
                   parse_constant=lambda c: (_ for _ in ()).throw(ValueError(c)))
    return _from_serde_json(v, "")


# ---------------------------------------------------------------------------
# serde_yaml 0.9 (YAML 1.2 core schema) -> Value -> PathAwareValue
# values.rs:287-366 (serde_yaml arm), used by guard-ffi run_checks' YAML fallback and by
# `cfn-guard test` spec inputs (commands/test.rs:480-484)
# ---------------------------------------------------------------------------
_Y12_INT = re.compile(r"^[-+]?(?:[0-9]+|0x[0-9a-fA-F]+|0o[0-7]+|0b[01]+)$")
_Y12_FLOAT = re.compile(r"^[-+]?(?:\.[0-9]+|[0-9]+(?:\.[0-9]*)?)(?:[eE][-+]?[0-9]+)?$")


def _y12_int(s):
    neg = s.startswith("-")
    body = s.lstrip("+-")
    if body.startswith("0x"):
        v = int(body[2:], 16)
    elif body.startswith("0o"):
        v = int(body[2:], 8)
    elif body.startswith("0b"):
        v = int(body[2:], 2)
    else:
        v = int(body)
    return -v if neg else v


def _serde_scalar(ev):
    val, tag, style = ev.value, ev.tag, ev.style
    if tag is not None and tag != "!":
        if tag.count("!") == 1 and tag.startswith("!"):
            fn = tag[1:]
            inner = PV(STRING, "", 0, 0, val)
            if fn in SINGLE_VALUE_FUNC_REF or fn in SEQUENCE_VALUE_FUNC_REF:
                return ("tagged", SHORT_FORM_TO_LONG[fn], inner)
            return inner
    if style != "":
        return PV(STRING, "", 0, 0, val)
    if val in ("~", "null", "Null", "NULL", ""):
        return PV(NULL, "", 0, 0)
    if val in ("true", "True", "TRUE"):
        return PV(BOOL, "", 0, 0, True)
    if val in ("false", "False", "FALSE"):
        return PV(BOOL, "", 0, 0, False)
    if _Y12_INT.match(val):
        v = _y12_int(val)
        if I64_MIN <= v <= I64_MAX:
            return PV(INT, "", 0, 0, v)
        if 0 <= v < (1 << 64):
            return PV(INT, "", 0, 0, v - (1 << 64))
        return PV(FLOAT, "", 0, 0, float(v))
    if _Y12_FLOAT.match(val):
        return PV(FLOAT, "", 0, 0, float(val))
    low = val.lower()
    if low in (".inf", "+.inf"):
        return PV(FLOAT, "", 0, 0, math.inf)
    if low == "-.inf":
        return PV(FLOAT, "", 0, 0, -math.inf)
    if low == ".nan":
        return PV(FLOAT, "", 0, 0, math.nan)
    return PV(STRING, "", 0, 0, val)


def load_serde_yaml_tree(content):
    """Returns a plain python tree: PV scalars, ('list', [...]), ('map', [(k, v)...]),
    ('tagged', fn, subtree)."""
    parser = CParser(content)
    stack = [[]]
    kinds = []
    tags = []
    while True:
        ev = parser.get_event()
        if ev is None:
            break
        name = type(ev).__name__
        if name == "ScalarEvent":
            stack[-1].append(_serde_scalar(ev))
        elif name in ("MappingStartEvent", "SequenceStartEvent"):
            stack.append([])
            kinds.append("map" if name == "MappingStartEvent" else "list")
            tags.append(ev.tag)
        elif name in ("MappingEndEvent", "SequenceEndEvent"):
            items = stack.pop()
            kind = kinds.pop()
            tag = tags.pop()
            if kind == "map":
                node = ("map", [(items[i], items[i + 1]) for i in range(0, len(items), 2)])
            else:
                node = ("list", items)
            if tag is not None and tag.count("!") == 1 and tag.startswith("!"):
                fn = tag[1:]
                if fn in SINGLE_VALUE_FUNC_REF or fn in SEQUENCE_VALUE_FUNC_REF:
                    node = ("tagged", SHORT_FORM_TO_LONG[fn], node)
            stack[-1].append(node)
        elif name == "AliasEvent":
            raise GuardError("YamlError", "aliases are outside the oracle's scope")
        elif name == "DocumentEndEvent":
            break
    return stack[0][0] if stack[0] else PV(NULL, "", 0, 0)


def serde_tree_to_pv(node, path=""):
    if isinstance(node, PV):
        return PV(node.kind, path, 0, 0, node.val)
    k = node[0]
    if k == "tagged":
        mv = MapValue()
        key = node[1]
        mv.keys.append(PV(STRING, path + "/" + key, 0, 0, key))
        mv.values[key] = serde_tree_to_pv(node[2], path + "/" + key)
        return PV(MAP, path, 0, 0, mv)
    if k == "list":
        return PV(LIST, path, 0, 0, [serde_tree_to_pv(e, "%s/%d" % (path, i)) for i, e in enumerate(node[1])])
    mv = MapValue()
    pairs = []
    for kn, vn in node[1]:
        if not isinstance(kn, PV) or kn.kind != STRING:
            raise GuardError("InternalError", "non string type detected for key in a map at , "
                             "cfn-guard only supports keys that are string types")
        if any(kn.val == k for k, _ in pairs):
            # serde_yaml 0.9 Mapping::deserialize: DuplicateKeyError (its position suffix not restated)
            raise GuardError("YamlError", "duplicate entry with key %s" % rust_debug_str(kn.val))
        pairs.append((kn.val, vn))
    for key, _ in pairs:
        mv.keys.append(PV(STRING, path + "/" + key, 0, 0, key))
    for key, vn in pairs:
        mv.values[key] = serde_tree_to_pv(vn, path + "/" + key)
    return PV(MAP, path, 0, 0, mv)


def pv_to_json_text(v):
    """Re-serialize a serde-mode PV as compact JSON text (lossless for ints/floats/strings)."""
    import json as _json
    def conv(x):
        if x.kind == MAP:
            return {k: conv(e) for k, e in x.val.values.items()}
        if x.kind == LIST:
            return [conv(e) for e in x.val]
        return x.val
    return _json.dumps(conv(v), ensure_ascii=False, allow_nan=False)
