"""PathAwareValue restatement (TEST INFRASTRUCTURE ONLY -- the parity oracle).

This module is part of the CPU oracle under ``oracle/``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker.  The product path never touches it.

It restates, in plain Python:
  * ``PathAwareValue``            guard/src/rules/path_value.rs:171-185
  * ``Path`` / ``Location`` Display path_value.rs:42-66
  * ``compare_values/compare_eq``  path_value.rs:1047-1152, ``compare_lt..ge`` 1154-1192
  * ``PartialEq`` (regex aware)    path_value.rs:245-291
  * serde ``Serialize``            path_value.rs:864-880, 480-588 (serde_json / ryu floats)
  * ``ValueOnlyDisplay``/Display   display.rs:33-107
  * derived ``Debug``              (Rust #[derive(Debug)] on PathAwareValue/Path/MapValue)
  * ``type_info``                  path_value.rs:985-1000
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

from .errors import GuardError
from . import rxcompat

# kinds
NULL, STRING, REGEX, BOOL, INT, FLOAT, CHAR, LIST, MAP, RANGE_INT, RANGE_FLOAT, RANGE_CHAR = (
    "Null", "String", "Regex", "Bool", "Int", "Float", "Char", "List", "Map",
    "RangeInt", "RangeFloat", "RangeChar")

LOWER_INCLUSIVE = 0x01
UPPER_INCLUSIVE = 0x02

TYPE_INFO = {
    NULL: "null", STRING: "String", REGEX: "Regex", BOOL: "bool", INT: "int",
    FLOAT: "float", CHAR: "char", LIST: "array", MAP: "map",
    RANGE_INT: "range(int, int)", RANGE_FLOAT: "range(float, float)",
    RANGE_CHAR: "range(char, char)",
}


class MapValue:
    """path_value.rs:130-164 -- ``keys`` keeps every key (duplicates too),
    ``values`` is an insertion-ordered map (IndexMap: last value, first position)."""

    __slots__ = ("keys", "values")

    def __init__(self):
        self.keys: List["PV"] = []
        self.values: Dict[str, "PV"] = {}


class PV:
    __slots__ = ("kind", "path", "line", "col", "val")

    def __init__(self, kind, path, line, col, val=None):
        self.kind = kind
        self.path = path
        self.line = line
        self.col = col
        self.val = val

    # -- helpers -----------------------------------------------------------
    def is_list(self):
        return self.kind == LIST

    def is_map(self):
        return self.kind == MAP

    def is_null(self):
        return self.kind == NULL

    def is_scalar(self):
        return self.kind not in (LIST, MAP)

    def type_info(self):
        return TYPE_INFO[self.kind]

    def path_display(self):
        # Path Display: "{pointer}[L:{line},C:{col}]"   path_value.rs:62-66
        return "%s[L:%d,C:%d]" % (self.path, self.line, self.col)

    def __eq__(self, other):  # PartialEq, path_value.rs:245-291
        return pv_eq(self, other)

    def __hash__(self):
        return 0

    def __repr__(self):
        return "PV(%s)" % display(self)


# ---------------------------------------------------------------------------
# float formatting
# ---------------------------------------------------------------------------
def _shortest(x: float):
    """Return (negative, digits, k): |x| == int(digits) * 10**k, digits w/o trailing zeros."""
    r = repr(abs(x))
    neg = math.copysign(1.0, x) < 0
    if "e" in r or "E" in r:
        mant, exp = r.lower().split("e")
        exp = int(exp)
    else:
        mant, exp = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    k = exp - len(fp)
    if not digits:
        return neg, "0", 0
    stripped = digits.rstrip("0")
    k += len(digits) - len(stripped)
    return neg, stripped, k


def rust_display_f64(x: float) -> str:
    """Rust ``impl Display for f64`` (shortest round-trip digits, never an exponent)."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    neg, d, k = _shortest(x)
    if d == "0":
        s = "0"
    elif k >= 0:
        s = d + "0" * k
    else:
        pos = len(d) + k
        if pos > 0:
            s = d[:pos] + "." + d[pos:]
        else:
            s = "0." + "0" * (-pos) + d
    return ("-" if neg else "") + s


def rust_debug_f64(x: float) -> str:
    """Rust ``impl Debug for f64``: decimal with >=1 fractional digit when
    1e-4 <= |x| < 1e16 (or zero), otherwise LowerExp shortest."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    ax = abs(x)
    neg, d, k = _shortest(x)
    sign = "-" if neg else ""
    if ax == 0.0 or (1e-4 <= ax < 1e16):
        s = rust_display_f64(ax)
        if "." not in s:
            s += ".0"
        return sign + s
    exp = len(d) - 1 + k
    mant = d[0] + ("." + d[1:] if len(d) > 1 else "")
    return "%s%se%d" % (sign, mant, exp)


def ryu_f64(x: float) -> str:
    """serde_json float output (ryu ``format64``)."""
    neg, d, k = _shortest(x)
    sign = "-" if neg else ""
    if d == "0":
        return sign + "0.0"
    length = len(d)
    kk = length + k
    if 0 <= k and kk <= 16:
        return sign + d + "0" * k + ".0"
    if 0 < kk <= 16:
        return sign + d[:kk] + "." + d[kk:]
    if -5 < kk <= 0:
        return sign + "0." + "0" * (-kk) + d
    if length == 1:
        return "%s%se%d" % (sign, d, kk - 1)
    return "%s%s.%se%d" % (sign, d[0], d[1:], kk - 1)


# ---------------------------------------------------------------------------
# Display (display.rs:33-107)
# ---------------------------------------------------------------------------
def _range_str(v, kind):
    lo, hi, inc = v
    f = (lambda z: rust_display_f64(z)) if kind == RANGE_FLOAT else (lambda z: str(z))
    return "%s%s,%s%s" % ("[" if inc & LOWER_INCLUSIVE else "(", f(lo), f(hi),
                          "]" if inc & UPPER_INCLUSIVE else ")")


def value_only(v: PV) -> str:
    k = v.kind
    if k == NULL:
        return '"NULL"'
    if k == STRING:
        return '"%s"' % v.val
    if k == REGEX:
        return '"/%s/"' % v.val
    if k == BOOL:
        return "true" if v.val else "false"
    if k == INT:
        return str(v.val)
    if k == FLOAT:
        return rust_display_f64(v.val)
    if k == CHAR:
        return "'%s'" % v.val
    if k == LIST:
        return "[" + ",".join(value_only(e) for e in v.val) + "]"
    if k == MAP:
        return "{" + ",".join('"%s":%s' % (key, value_only(e)) for key, e in v.val.values.items()) + "}"
    return _range_str(v.val, k)


def display(v: PV) -> str:
    return "Path=%s Value=%s" % (v.path_display(), value_only(v))


def display_path_only(v: PV) -> str:
    """`self_path().0` -- the JSON pointer alone (display.rs:157-160)"""
    return v.path


# ---------------------------------------------------------------------------
# Rust Debug (derived)
# ---------------------------------------------------------------------------
def rust_debug_str(s: str) -> str:
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
        elif ch == "\0":
            out.append("\\0")
        elif o < 0x20 or o == 0x7F or (0x80 <= o < 0xA0):
            out.append("\\u{%x}" % o)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _debug_path(v: PV) -> str:
    return 'Path(%s, Location { line: %d, col: %d })' % (rust_debug_str(v.path), v.line, v.col)


def rust_debug(v: PV) -> str:
    k = v.kind
    p = _debug_path(v)
    if k == NULL:
        return "Null(%s)" % p
    if k in (STRING, REGEX):
        return "%s((%s, %s))" % (k, p, rust_debug_str(v.val))
    if k == BOOL:
        return "Bool((%s, %s))" % (p, "true" if v.val else "false")
    if k == INT:
        return "Int((%s, %d))" % (p, v.val)
    if k == FLOAT:
        return "Float((%s, %s))" % (p, rust_debug_f64(v.val))
    if k == CHAR:
        return "Char((%s, %s))" % (p, _debug_char(v.val))
    if k == LIST:
        return "List((%s, [%s]))" % (p, ", ".join(rust_debug(e) for e in v.val))
    if k == MAP:
        keys = ", ".join(rust_debug(e) for e in v.val.keys)
        vals = ", ".join("%s: %s" % (rust_debug_str(key), rust_debug(e)) for key, e in v.val.values.items())
        return "Map((%s, MapValue { keys: [%s], values: {%s} }))" % (p, keys, vals)
    lo, hi, inc = v.val
    f = rust_debug_f64 if k == RANGE_FLOAT else (_debug_char if k == RANGE_CHAR else str)
    return "%s((%s, RangeType { upper: %s, lower: %s, inclusive: %d }))" % (k, p, f(hi), f(lo), inc)


def _debug_char(c):
    if c == "'":
        return "'\\''"
    s = rust_debug_str(c)[1:-1]
    if s == '\\"':
        s = '"'
    return "'%s'" % s


# ---------------------------------------------------------------------------
# serde serialization -> python JSON tree (floats tagged for ryu printing)
# ---------------------------------------------------------------------------
class JFloat:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v


def to_json_value(v: PV):
    k = v.kind
    if k == NULL:
        return None
    if k == STRING:
        return v.val
    if k == REGEX:
        return "/%s/" % v.val
    if k == BOOL:
        return bool(v.val)
    if k == INT:
        return int(v.val)
    if k == FLOAT:
        if math.isnan(v.val) or math.isinf(v.val):
            raise GuardError("IncompatibleError",
                             "Could not convert float %s to serde::Value::Number" % rust_display_f64(v.val))
        return JFloat(v.val)
    if k == CHAR:
        return v.val
    if k == LIST:
        return [to_json_value(e) for e in v.val]
    if k == MAP:
        d = {}
        for key, e in v.val.values.items():
            d[key] = to_json_value(e)
        return d
    lo, hi, inc = v.val
    return _range_str(v.val, k) if k != RANGE_FLOAT else _range_str(v.val, k)


def serialize(v: PV):
    """PathAwareValue Serialize: {"path": ..., "value": ...}"""
    return {"path": v.path, "value": to_json_value(v)}


# ---------------------------------------------------------------------------
# comparisons
# ---------------------------------------------------------------------------
class NotComparable(GuardError):
    def __init__(self, msg):
        GuardError.__init__(self, "NotComparable", msg)


def _cmp(a, b):
    return (a > b) - (a < b)


def _str_cmp(a: str, b: str):
    # Rust String Ord is bytewise on UTF-8
    ab, bb = a.encode("utf-8", "surrogatepass"), b.encode("utf-8", "surrogatepass")
    return _cmp(ab, bb)


def compare_values(a: PV, b: PV) -> int:
    ka, kb = a.kind, b.kind
    if ka == NULL and kb == NULL:
        return 0
    if ka == INT and kb == INT:
        return _cmp(a.val, b.val)
    if ka == STRING and kb == STRING:
        return _str_cmp(a.val, b.val)
    if ka == FLOAT and kb == FLOAT:
        if math.isnan(a.val) or math.isnan(b.val):
            raise NotComparable("Float values are not comparable")
        return _cmp(a.val, b.val)
    if ka == CHAR and kb == CHAR:
        return _cmp(ord(a.val), ord(b.val))
    raise NotComparable("PathAwareValues are not comparable %s, %s" % (a.type_info(), b.type_info()))


def is_within(rng, x, key=lambda z: z):
    lo, hi, inc = rng
    lower = key(lo) <= key(x) if inc & LOWER_INCLUSIVE else key(lo) < key(x)
    upper = key(hi) >= key(x) if inc & UPPER_INCLUSIVE else key(hi) > key(x)
    return lower and upper


def regex_is_match(pattern: str, s: str) -> bool:
    return rxcompat.is_match(pattern, s)


def compare_eq(a: PV, b: PV) -> bool:
    ka, kb = a.kind, b.kind
    if ka == STRING and kb == REGEX:
        return regex_is_match(b.val, a.val)
    if ka == REGEX and kb == STRING:
        return regex_is_match(a.val, b.val)
    if ka == STRING and kb == STRING:
        return a.val == b.val
    if ka == MAP and kb == MAP:
        m1, m2 = a.val.values, b.val.values
        if len(m1) != len(m2):
            return False
        for key, v1 in m1.items():
            v2 = m2.get(key)
            if v2 is None:
                return False
            if not compare_eq(v1, v2):
                return False
        return True
    if ka == LIST and kb == LIST:
        if len(a.val) != len(b.val):
            return False
        for x, y in zip(a.val, b.val):
            if not compare_eq(x, y):
                return False
        return True
    if ka == BOOL and kb == BOOL:
        return a.val == b.val
    if ka == REGEX and kb == REGEX:
        return a.val == b.val
    if ka == INT and kb == RANGE_INT:
        return is_within(b.val, a.val)
    if ka == FLOAT and kb == RANGE_FLOAT:
        return is_within(b.val, a.val)
    if ka == CHAR and kb == RANGE_CHAR:
        return is_within(b.val, a.val, key=ord)
    return compare_values(a, b) == 0


def pv_eq(a: PV, b: PV) -> bool:
    """PartialEq for PathAwareValue (path_value.rs:245-291): errors => false."""
    ka, kb = a.kind, b.kind
    if ka == MAP and kb == MAP:
        m1, m2 = a.val.values, b.val.values
        if len(m1) != len(m2):
            return False
        for key, v1 in m1.items():
            v2 = m2.get(key)
            if v2 is None or not pv_eq(v1, v2):
                return False
        return True
    if ka == LIST and kb == LIST:
        return len(a.val) == len(b.val) and all(pv_eq(x, y) for x, y in zip(a.val, b.val))
    if ka == BOOL and kb == BOOL:
        return a.val == b.val
    if ka == STRING and kb == REGEX:
        return regex_is_match(b.val, a.val)
    if ka == REGEX and kb == STRING:
        return regex_is_match(a.val, b.val)
    if ka == REGEX and kb == REGEX:
        return a.val == b.val
    if ka == INT and kb == RANGE_INT:
        return is_within(b.val, a.val)
    if ka == FLOAT and kb == RANGE_FLOAT:
        return is_within(b.val, a.val)
    if ka == CHAR and kb == RANGE_CHAR:
        return is_within(b.val, a.val, key=ord)
    try:
        return compare_values(a, b) == 0
    except GuardError:
        return False


def compare_lt(a, b):
    return compare_values(a, b) < 0


def compare_le(a, b):
    return compare_values(a, b) <= 0


def compare_gt(a, b):
    return compare_values(a, b) > 0


def compare_ge(a, b):
    return compare_values(a, b) >= 0


# ---------------------------------------------------------------------------
# constructors
# ---------------------------------------------------------------------------
def from_value(value, path="", line=0, col=0) -> PV:
    """PathAwareValue::try_from((&Value, Path)) -- path_value.rs:371-406.
    ``value`` is a parser literal: ('kind', payload) tuples from parser.py."""
    kind, payload = value
    if kind == LIST:
        return PV(LIST, path, line, col,
                  [from_value(e, "%s/%d" % (path, i), line, col) for i, e in enumerate(payload)])
    if kind == MAP:
        mv = MapValue()
        for key, _ in payload:
            mv.keys.append(PV(STRING, path + "/" + key, line, col, key))
        for key, e in payload:
            mv.values[key] = from_value(e, path + "/" + key, line, col)
        return PV(MAP, path, line, col, mv)
    return PV(kind, path, line, col, payload)


# ---------------------------------------------------------------------------
# PathAwareValue::merge (path_value.rs:889-919), used by `validate -i` (validate.rs:317-350,
# structured.rs:51-65)
# ---------------------------------------------------------------------------
def merge(this: PV, other: PV) -> PV:
    """``self.merge(other)`` on a copy of ``this`` (the caller's value is left unchanged, as the
    reference merges ``data.clone()``)."""
    if this.kind == LIST and other.kind == LIST:
        return PV(LIST, this.path, this.line, this.col, list(this.val) + list(other.val))
    if this.kind == MAP and other.kind == MAP:
        mv = MapValue()
        mv.keys = list(this.val.keys)
        mv.values = dict(this.val.values)
        for key, value in other.val.values.items():
            if key in mv.values:
                raise GuardError("MultipleValues", "Key %s, already exists in map" % key)
            mv.values[key] = value
            # map.keys.push(String((path.extend_str(&key), key))): other's path + "/key", other's location
            mv.keys.append(PV(STRING, other.path + "/" + key, other.line, other.col, key))
        return PV(MAP, this.path, this.line, this.col, mv)
    raise GuardError("IncompatibleError", "Types are not compatible for merges %s, %s"
                     % (this.type_info(), other.type_info()))
