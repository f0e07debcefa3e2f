"""Guard DSL parser restatement (TEST INFRASTRUCTURE ONLY -- the parity oracle).

A PEG restatement of the nom 7.1.3 grammar in ``guard/src/rules/parser.rs`` (function names
below follow the reference's combinators 1:1, with their file:line).  ``Err`` models
``nom::Err::Error`` (recoverable, ``alt`` tries the next branch) and ``Fail`` models
``nom::Err::Failure`` (raised by ``cut``).  Both carry nom's ParserError payload (the input
position the failing combinator saw, and its context), propagated as nom 7.1.3 does: ``alt``
reports its last alternative's error, ``many1`` / ``separated_list`` their element's,
``fold_many1`` a fresh error at its own input, ``context`` its input position and "ctx/inner",
``cut`` turns Error into Failure.  A failed parse raises ``GuardError('ParseError', "Parsing Error
Error parsing file F at line L at column C, when handling CTX, fragment REST")`` as
``errors.rs:107-115`` / ``parser.rs:88-101`` display it.

AST nodes are plain dicts/tuples mirroring ``guard/src/rules/exprs.rs``.
"""
from .errors import GuardError
from . import pv as P
from . import rxcompat


class Err(Exception):
    def __init__(self, pos=0, ctx=""):
        super().__init__(pos, ctx)
        self.pos, self.ctx = pos, ctx


class Fail(Exception):
    def __init__(self, pos=0, ctx=""):
        super().__init__(pos, ctx)
        self.pos, self.ctx = pos, ctx


def _add_ctx(ctx, inner):
    """nom ContextError::add_context (parser.rs:48-62)"""
    return ctx if not inner else "%s/%s" % (ctx, inner)


CTX_CMP = "expecting comparison binary operators like >, <= or unary operators KEYS, EXISTS, EMPTY or NOT"
CTX_RHS = 'expecting either a property access "engine.core" or value like "string" or ["this", "that"]'


FUNCTION_ARITY = {
    "count": 1, "join": 2, "json_parse": 1, "now": 0, "parse_boolean": 1, "parse_char": 1,
    "parse_epoch": 1, "parse_float": 1, "parse_int": 1, "parse_string": 1,
    "regex_replace": 3, "substring": 3, "to_lower": 1, "to_upper": 1, "url_decode": 1,
}

MULTISPACE = " \t\r\n"


class Parser:
    def __init__(self, text, file_name):
        self.s = text
        self.n = len(text)
        self.file = file_name
        self.line_starts = [0]
        for i, ch in enumerate(text):
            if ch == "\n":
                self.line_starts.append(i + 1)

    # -- location -------------------------------------------------------------
    def loc(self, p, utf8=True):
        import bisect
        li = bisect.bisect_right(self.line_starts, p) - 1
        start = self.line_starts[li]
        if utf8:
            col = p - start + 1  # python str index == char index
        else:
            col = len(self.s[start:p].encode("utf-8")) + 1
        return {"line": li + 1, "column": col, "file": self.file}

    def error_text(self, p, ctx):
        """ParserError Display (parser.rs:88-101)"""
        lc = self.loc(p)
        return "Error parsing file %s at line %d at column %d, when handling %s, fragment %s" % (
            self.file, lc["line"], lc["column"], ctx, self.s[p:])

    # -- primitives -----------------------------------------------------------
    def tag(self, p, t):
        if self.s.startswith(t, p):
            return p + len(t)
        raise Err(p)

    def char(self, p, c):
        if p < self.n and self.s[p] == c:
            return p + 1
        raise Err(p)

    def multispace0(self, p):
        while p < self.n and self.s[p] in MULTISPACE:
            p += 1
        return p

    def space0(self, p):
        while p < self.n and self.s[p] in " \t":
            p += 1
        return p

    def space1(self, p):
        q = self.space0(p)
        if q == p:
            raise Err(p)
        return q

    def digit1(self, p):
        q = p
        while q < self.n and "0" <= self.s[q] <= "9":
            q += 1
        if q == p:
            raise Err(p)
        return q

    def alpha1(self, p):
        q = p
        while q < self.n and (("a" <= self.s[q] <= "z") or ("A" <= self.s[q] <= "Z")):
            q += 1
        if q == p:
            raise Err(p)
        return q

    # comment2  parser.rs:111-113
    def comment2(self, p):
        p = self.char(p, "#")
        while p < self.n and self.s[p] != "\n":
            p += 1
        return self.multispace0(p)

    def white_space_or_comment(self, p):
        q = self.multispace0(p)
        if q > p:
            return q
        return self.comment2(p)

    def zero_or_more_ws_or_comment(self, p):
        while True:
            try:
                q = self.white_space_or_comment(p)
            except Err:
                return p
            if q == p:
                return p
            p = q

    def one_or_more_ws_or_comment(self, p):
        q = self.white_space_or_comment(p)
        return self.zero_or_more_ws_or_comment(q)

    def white_space(self, p, ch):
        return self.char(self.zero_or_more_ws_or_comment(p), ch)

    # -- values  parser.rs:165-455 ------------------------------------------
    def parse_int_value(self, p):
        try:
            q = self.digit1(p)
            v = int(self.s[p:q])
            if v > (1 << 63) - 1:
                raise Err(p)   # map_res: the error is at map_res's input
            return q, ("Int", v)
        except Err:
            pass
        q = self.tag(p, "-")
        r = self.digit1(q)
        v = int(self.s[q:r])
        if v > (1 << 63) - 1:
            raise Err(p)
        return r, ("Int", -v)

    def parse_string_inner(self, p, ch):
        p = self.char(p, ch)
        start_input = p
        completed = []
        span = p
        while True:
            q = span
            while q < self.n and self.s[q] != ch:
                q += 1
            frag = self.s[span:q]
            if frag.endswith("\\"):
                completed.append(frag[:-1])
                completed.append(ch)
                if q >= self.n:
                    raise Err(start_input, "Could not parse string")
                span = q + 1
                continue
            completed.append(frag)
            if q >= self.n or self.s[q] != ch:
                raise Fail(q)   # cut(char(ch))
            return q + 1, ("String", "".join(completed))

    def parse_string(self, p):
        try:
            return self.parse_string_inner(p, "'")
        except Err:
            return self.parse_string_inner(p, '"')

    def parse_bool(self, p):
        for t, v in (("true", True), ("True", True), ("false", False), ("False", False)):
            if self.s.startswith(t, p):
                return p + len(t), ("Bool", v)
        raise Err(p)

    def _recognize_float(self, p):
        # nom::number::complete::recognize_float (+ nan/inf exceptions)
        q = p
        if q < self.n and self.s[q] in "+-":
            q += 1
        if q < self.n and "0" <= self.s[q] <= "9":
            q = self.digit1(q)
            if q < self.n and self.s[q] == ".":
                q += 1
                while q < self.n and "0" <= self.s[q] <= "9":
                    q += 1
        elif q < self.n and self.s[q] == "." and q + 1 < self.n and "0" <= self.s[q + 1] <= "9":
            q = self.digit1(q + 1)
        else:
            raise Err(p)
        if q < self.n and self.s[q] in "eE":
            r = q + 1
            if r < self.n and self.s[r] in "+-":
                r += 1
            try:
                r = self.digit1(r)
            except Err as e:
                raise Fail(e.pos, e.ctx)   # cut(digit1)
            q = r
        return q

    def parse_float(self, p):
        whole = self.digit1(p)
        q = whole
        frac = False
        if q < self.n and self.s[q] == ".":
            try:
                q = self.digit1(q + 1)
                frac = True
            except Err:
                q = whole
        expo = False
        if q < self.n and self.s[q] in "eE" and q + 1 < self.n and self.s[q + 1] in "+-":
            try:
                self.digit1(q + 2)
                expo = True
            except Err:
                pass
        if frac or expo:
            r = self._recognize_float(p)
            return r, ("Float", float(self.s[p:r]))
        raise Err(p, "Could not parse floating number")

    def parse_regex_inner(self, p):
        regex = []
        span = p
        while True:
            q = span
            while q < self.n and self.s[q] != "/":
                q += 1
            if q == span:
                raise Err(span)   # is_not("/")
            frag = self.s[span:q]
            if frag.endswith("\\"):
                regex.append(frag[:-1])
                regex.append("/")
                if q >= self.n:
                    raise Err(p, "Could not parse regular expression")
                span = q + 1
                continue
            regex.append(frag)
            rx = "".join(regex)
            if not rxcompat.is_valid(rx):
                # the reference appends fancy-regex's error text; the alternatives around a regex
                # literal always report a later alternative's error, so it never reaches a message
                raise Err(p, "Could not parse regular expression")
            return q, ("Regex", rx)

    def parse_regex(self, p):
        p = self.char(p, "/")
        q, v = self.parse_regex_inner(p)
        q = self.char(q, "/")
        return q, v

    def parse_char(self, p):
        if p < self.n:
            return p + 1, ("Char", self.s[p])
        raise Err(p)

    def range_value(self, p):
        p = self.space0(p)
        for f in (self.parse_float, self.parse_int_value):
            try:
                q, v = f(p)
                return self.space0(q), v
            except Err:
                continue
        q, v = self.parse_char(p)
        return self.space0(q), v

    def parse_range(self, p):
        p = self.char(p, "r")
        if p < self.n and self.s[p] in "([":
            open_ = self.s[p]
            p += 1
        else:
            raise Err(p)
        p, a = self.range_value(p)
        p = self.char(p, ",")
        p, b = self.range_value(p)
        if p < self.n and self.s[p] in ")]":
            close = self.s[p]
            p += 1
        else:
            raise Err(p)
        inc = (P.LOWER_INCLUSIVE if open_ == "[" else 0) | (P.UPPER_INCLUSIVE if close == "]" else 0)
        if a[0] == "Int" and b[0] == "Int":
            return p, ("RangeInt", (a[1], b[1], inc))
        if a[0] == "Float" and b[0] == "Float":
            return p, ("RangeFloat", (a[1], b[1], inc))
        if a[0] == "Char" and b[0] == "Char":
            return p, ("RangeChar", (a[1], b[1], inc))
        raise Fail(p, "Could not parse range")

    def parse_scalar_value(self, p):
        for f in (self.parse_string, self.parse_float, self.parse_int_value, self.parse_bool):
            try:
                return f(p)
            except Err:
                continue
        return self.parse_regex(p)   # alt: the last alternative's error

    def separated_list0(self, p, sep, elem):
        out = []
        try:
            p, v = elem(p)
        except Err:
            return p, out
        out.append(v)
        while True:
            try:
                q = sep(p)
            except Err:
                return p, out
            try:
                q, v = elem(q)
            except Err:
                return p, out
            out.append(v)
            p = q

    def separated_list1(self, p, sep, elem):
        p, v = elem(p)
        out = [v]
        while True:
            try:
                q = sep(p)
            except Err:
                return p, out
            try:
                q, v = elem(q)
            except Err:
                return p, out
            out.append(v)
            p = q

    def parse_list(self, p):
        p = self.white_space(p, "[")
        p, items = self.separated_list0(p, lambda q: self.white_space(q, ","), self.parse_value)
        p = self.white_space(p, "]")
        return p, ("List", items)

    def key_part(self, p):
        q = p
        while q < self.n and (self.s[q].isalnum() or self.s[q] in "-_"):
            q += 1
        if q > p:
            return q, self.s[p:q]
        q, v = self.parse_string(p)
        return q, v[1]

    def key_value(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        p, k = self.key_part(p)
        p = self.white_space(p, ":")
        p, v = self.parse_value(p)
        return p, (k, v)

    def parse_map(self, p):
        p = self.char(p, "{")
        p, kvs = self.separated_list0(p, lambda q: self.white_space(q, ","), self.key_value)
        p = self.white_space(p, "}")
        d = []
        for k, v in kvs:  # IndexMap collect: last value wins, first position
            for i, (k2, _) in enumerate(d):
                if k2 == k:
                    d[i] = (k, v)
                    break
            else:
                d.append((k, v))
        return p, ("Map", d)

    def parse_null(self, p):
        for t in ("null", "NULL"):
            if self.s.startswith(t, p):
                return p + len(t), ("Null", None)
        raise Err(p)

    def parse_value(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        for f in (self.parse_null, self.parse_scalar_value, self.parse_range, self.parse_list):
            try:
                return f(p)
            except Err:
                continue
        return self.parse_map(p)

    # -- expressions ----------------------------------------------------------
    def var_name(self, p):
        q = self.alpha1(p)
        while q < self.n and (self.s[q].isalnum() or self.s[q] == "_"):
            q += 1
        return q, self.s[p:q]

    def var_name_access_inclusive(self, p):
        p = self.char(p, "%")
        q, name = self.var_name(p)
        return q, "%" + name

    def in_keyword(self, p):
        for t in ("in", "IN"):
            if self.s.startswith(t, p):
                return p + len(t), "In"
        raise Err(p)

    def not_(self, p):
        for t in ("not", "NOT"):
            if self.s.startswith(t, p):
                try:
                    return self.space1(p + len(t))
                except Err:
                    pass
        return self.char(p, "!")

    def eq(self, p):
        if self.s.startswith("==", p):
            return p + 2, ("Eq", False)
        if self.s.startswith("!=", p):
            return p + 2, ("Eq", True)
        raise Err(p)

    _UNARY_WORDS = [
        (("EXISTS", "exists"), "Exists"), (("EMPTY", "empty"), "Empty"),
    ]
    _IS_TYPES = [
        (("IS_STRING", "is_string"), "IsString"), (("IS_LIST", "is_list"), "IsList"),
        (("IS_STRUCT", "is_struct"), "IsMap"), (("IS_BOOL", "is_bool"), "IsBool"),
        (("IS_INT", "is_int"), "IsInt"), (("IS_NULL", "is_null"), "IsNull"),
        (("IS_FLOAT", "is_float"), "IsFloat"),
    ]

    def other_operations(self, p):
        neg = False
        try:
            p = self.not_(p)
            neg = True
        except Err:
            pass
        try:
            q, op = self.in_keyword(p)
            return q, (op, neg)
        except Err:
            pass
        for words, op in self._UNARY_WORDS + self._IS_TYPES:
            for w in words:
                if self.s.startswith(w, p):
                    return p + len(w), (op, neg)
        raise Err(p)

    def value_cmp(self, p):
        if self.s.startswith("<<", p):
            raise Err(p, "Custom message tag detected")
        try:
            return self.eq(p)
        except Err:
            pass
        for t, op in ((">=", "Ge"), ("<=", "Le"), (">", "Gt"), ("<", "Lt")):
            if self.s.startswith(t, p):
                return p + len(t), (op, False)
        return self.other_operations(p)

    def custom_message(self, p):
        p = self.tag(p, "<<")
        j = self.s.find(">>", p)
        if j < 0:
            raise Fail(p, "Unable to find a closing >> tag for message")
        return j + 2, self.s[p:j]

    def variable_capture_in_map_or_index(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        p, var = self.var_name(p)
        p = self.space0(p)
        p = self.char(p, "|")
        return p, var

    def open_array(self, p):
        return self.white_space(p, "[")

    def close_array(self, p):
        return self.white_space(p, "]")

    def cut(self, f, *a):
        try:
            return f(*a)
        except Err as e:
            raise Fail(e.pos, e.ctx)

    def opt(self, f, p):
        try:
            return f(p)
        except Err:
            return None

    def predicate_filter_clauses(self, p):
        p = self.open_array(p)
        r = self.opt(self.variable_capture_in_map_or_index, p)
        var = None
        if r is not None:
            p, var = r
        p, conj = self.cnf_clauses(p, self.clause)
        p = self.cut(self.close_array, p)
        return p, ("Filter", var, conj)

    def dotted_property(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        p = self.char(p, ".")
        try:
            q, v = self.parse_int_value(p)
            return q, ("Index", _i32(v[1]))
        except Err:
            pass
        try:
            q, name = self.property_name(p)
            return q, ("Key", name)
        except Err:
            pass
        try:
            q, name = self.var_name_access_inclusive(p)
            return q, ("Key", name)
        except Err:
            pass
        q = self.char(p, "*")
        return q, ("AllValues", None)

    def all_indices(self, p):
        p = self.open_array(p)
        q = self.zero_or_more_ws_or_comment(p)
        if q < self.n and self.s[q] == "*":
            part, p = ("AllIndices", None), q + 1
        else:
            p, name = self.var_name(p)
            part = ("AllIndices", name)
        p = self.close_array(p)
        return p, part

    def array_index(self, p):
        p = self.open_array(p)
        p, v = self.parse_int_value(p)
        p = self.cut(self.close_array, p)
        return p, ("Index", _i32(v[1]))

    def map_key_lookup(self, p):
        p = self.open_array(p)
        try:
            q, v = self.parse_string(p)
            part = ("Key", v[1])
        except Err:
            q = self.zero_or_more_ws_or_comment(p)
            q, name = self.var_name(q)
            q = self.zero_or_more_ws_or_comment(q)
            part = ("AllValues", name)
        q = self.close_array(q)
        return q, part

    def map_keys_match(self, p):
        p = self.open_array(p)
        r = self.opt(self.variable_capture_in_map_or_index, p)
        var = None
        if r is not None:
            p, var = r
        p = self.zero_or_more_ws_or_comment(p)
        for t in ("KEYS", "keys"):
            if self.s.startswith(t, p):
                p += len(t)
                break
        else:
            raise Err(p)

        def cmp_(q):
            q = self.zero_or_more_ws_or_comment(q)
            try:
                return self.eq(q)
            except Err:
                pass
            try:
                r2, _ = self.in_keyword(q)
                return r2, ("In", False)
            except Err:
                pass
            q = self.not_(q)
            r2, _ = self.in_keyword(q)
            return r2, ("In", True)

        p, cmp = self.cut(cmp_, p)

        def with_(q):
            q = self.zero_or_more_ws_or_comment(q)
            try:
                r2, v = self.parse_value(q)
                return r2, ("Value", P.from_value(_lit(v)))
            except Err:
                pass
            q = self.zero_or_more_ws_or_comment(q)
            r2, acc = self.access(q)
            return r2, ("Access", acc)

        p, with_v = self.cut(with_, p)
        p = self.close_array(p)
        return p, ("MapKeyFilter", var, {"comparator": cmp, "compare_with": with_v})

    def predicate_or_index(self, p):
        for f in (self.all_indices, self.array_index, self.map_key_lookup, self.map_keys_match):
            try:
                return f(p)
            except Err:
                continue
        return self.predicate_filter_clauses(p)

    def dotted_access(self, p):
        def one(q):
            try:
                return self.dotted_property(q)
            except Err:
                return self.predicate_or_index(q)
        try:
            p, v = one(p)
        except Err:
            raise Err(p)   # fold_many1: from_error_kind(input, Many1)
        out = [v]
        while True:
            try:
                q, v = one(p)
            except Err:
                return p, out
            out.append(v)
            p = q

    def property_name(self, p):
        try:
            return self.var_name(p)
        except Err:
            q, v = self.parse_string(p)
            return q, v[1]

    def some_keyword(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        for t in ("SOME", "some"):
            if self.s.startswith(t, p):
                return self.one_or_more_ws_or_comment(p + len(t))
        raise Err(p)

    def this_keyword(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        for t in ("this", "THIS"):
            if self.s.startswith(t, p):
                return p + len(t), ("This",)
        raise Err(p)

    def access(self, p):
        r = self.opt(self.some_keyword, p)
        some = r is not None
        if some:
            p = r
        try:
            p, first = self.this_keyword(p)
        except Err:
            try:
                p, name = self.var_name_access_inclusive(p)
            except Err:
                p, name = self.property_name(p)
            first = ("Key", name)
        r = self.opt(self.dotted_access, p)
        if r is not None:
            p, parts = r
            parts.insert(0, first)
            if _is_variable(first):
                if not (len(parts) > 1 and parts[1][0] == "AllIndices"):
                    parts.insert(1, ("AllIndices", None))
            query = parts
        else:
            query = [first]
        return p, {"query": query, "match_all": not some}

    def clause_with_map(self, p, kind):
        location = self.loc(p)
        p = self.zero_or_more_ws_or_comment(p)
        negation = False
        try:
            p = self.not_(p)
            negation = True
        except Err:
            pass
        p, query = self.access(p)
        p = self.zero_or_more_ws_or_comment(p)
        try:
            p, cmp = self.value_cmp(p)
        except Err as e:   # context(.., value_cmp)  parser.rs:974
            raise Err(p, _add_ctx(CTX_CMP, e.ctx))
        if cmp[0] in UNARY_OPS:
            q = self.zero_or_more_ws_or_comment(p)
            msg = None
            try:
                p, msg = self.custom_message(q)
            except Err:
                p = q
            return p, {"kind": kind, "query": query, "comparator": cmp, "compare_with": None,
                       "custom_message": msg, "location": location, "negation": negation}

        def with_msg(r):
            q = self.zero_or_more_ws_or_comment(r)
            try:
                return self.custom_message(q)
            except Err:
                return q, None

        def rhs(q):
            try:
                r, v = self.parse_value(q)
                v = ("Value", P.from_value(_lit(v)))
                r, m = with_msg(r)
                return r, (v, m)
            except Err:
                pass
            try:
                r = self.zero_or_more_ws_or_comment(q)
                r, f = self.function_expr(r)
                r, m = with_msg(r)
                return r, (("Func", f), m)
            except Err:
                pass
            r = self.zero_or_more_ws_or_comment(q)
            r, acc = self.access(r)
            r, m = with_msg(r)
            return r, (("Access", acc), m)

        # context(.., cut(alt(...)))  parser.rs:1000-1023
        try:
            p, (with_v, msg) = self.cut(rhs, p)
        except Fail as e:
            raise Fail(p, _add_ctx(CTX_RHS, e.ctx))
        return p, {"kind": kind, "query": query, "comparator": cmp, "compare_with": with_v,
                   "custom_message": msg, "location": location, "negation": negation}

    def block_clause(self, p):
        location = self.loc(p)
        p, query = self.access(p)
        not_empty = False
        try:
            q = self.zero_or_more_ws_or_comment(p)
            q = self.not_(q)
            q = self.tag_any(q, ("EMPTY", "empty"))
            p, not_empty = q, True
        except Err:
            pass
        p, (assigns, conj) = self.block(p, self.clause)
        return p, {"kind": "BlockClause", "query": query, "block": {"assignments": assigns, "conjunctions": conj},
                   "location": location, "not_empty": not_empty}

    def tag_any(self, p, tags):
        for t in tags:
            if self.s.startswith(t, p):
                return p + len(t)
        raise Err(p)

    def function_expr(self, p):
        location = self.loc(p, utf8=False)
        p, (name, params) = self.call_expr(p)
        # parser.rs:1082-1100, errors at the input after the call
        if name not in FUNCTION_ARITY:
            raise Err(p, "Parser Error when parsing `No function with the name '%s' exists.`" % name)
        if len(params) != FUNCTION_ARITY[name]:
            raise Err(p, "function: %s requires: %d parameters to be passed, but received: %d"
                      % (name, FUNCTION_ARITY[name], len(params)))
        return p, {"name": name, "parameters": params, "location": location}

    def let_value(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        try:
            q, v = self.parse_value(p)
            return q, ("Value", P.from_value(_lit(v)))
        except Err:
            pass
        try:
            q, f = self.function_expr(p)
            return q, ("Func", f)
        except Err:
            pass
        q, acc = self.access(p)
        return q, ("Access", acc)

    def call_expr(self, p):
        p, name = self.var_name(p)
        p = self.char(p, "(")

        def elem(q):
            q = self.multispace0(q)
            q, v = self.let_value(q)
            return self.multispace0(q), v

        p, params = self.separated_list0(p, lambda q: self.char(q, ","), elem)
        p = self.char(p, ")")
        return p, (name, params)

    def parameterized_rule_call_clause(self, p):
        location = self.loc(p)
        negation = False
        try:
            p = self.not_(p)
            negation = True
        except Err:
            pass
        p, (name, params) = self.call_expr(p)
        msg = None
        try:
            q = self.zero_or_more_ws_or_comment(p)
            p, msg = self.custom_message(q)
        except Err:
            pass
        return p, {"kind": "ParamRule", "parameters": params,
                   "named_rule": {"dependent_rule": name, "negation": negation, "custom_message": msg,
                                  "location": location}}

    def clause(self, p):
        try:
            return self.when_block(p, self.single_clauses, self.clause)
        except Err:
            pass
        try:
            return self.block_clause(p)
        except Err:
            pass
        try:
            return self.parameterized_rule_call_clause(p)
        except Err:
            pass
        return self.clause_with_map(p, "Clause")

    def single_clause(self, p):
        return self.clause_with_map(p, "Clause")

    def newline(self, p):
        for t in ("\n", "\r\n"):
            if self.s.startswith(t, p):
                return p + len(t)
        raise Err(p)

    def rule_clause(self, p):
        location = self.loc(p)
        negation = False
        try:
            p = self.not_(p)
            negation = True
        except Err:
            pass
        p, name = self.var_name(p)
        do_return = p >= self.n
        if not do_return:
            for f in (lambda q: self.newline(self.space0(q)),
                      lambda q: self.comment2(self.space0(q)),
                      lambda q: self.char(self.space0(q), "{"),
                      self.or_join):
                try:
                    f(p)
                    do_return = True
                    break
                except Err:
                    continue
        if do_return:
            return p, {"kind": "NamedRule", "dependent_rule": name, "location": location,
                       "negation": negation, "custom_message": None}
        p, msg = self.cut(lambda q: self.custom_message(self.space0(q)), p)
        return p, {"kind": "NamedRule", "dependent_rule": name, "location": location,
                   "negation": negation, "custom_message": msg}

    def cnf_clauses(self, p, f):
        conj = []
        p0 = p
        while True:
            try:
                p2, disj = self.disjunction_clauses(p, f)
            except Err:
                if not conj:   # parser.rs:1300-1312
                    lc = self.loc(p0)
                    raise Fail(p0, "There were no clauses present %s#%d@%d" % (self.file, lc["line"], lc["column"]))
                return p, conj
            p = p2
            conj.append(disj)

    def disjunction_clauses(self, p, f):
        def elem(q):
            return f(self.zero_or_more_ws_or_comment(q))
        return self.separated_list1(p, self.or_join, elem)

    def single_clauses(self, p):
        def f(q):
            try:
                return self.single_clause(q)
            except Err:
                pass
            try:
                return self.parameterized_rule_call_clause(q)
            except Err:
                pass
            return self.rule_clause(q)
        return self.cnf_clauses(p, f)

    def clause_or_rule_clause(self, p):
        try:
            return self.clause(p)
        except Err:
            return self.rule_clause(p)

    def let_assignment_expr(self, p):
        p = self.tag(p, "let")
        p = self.one_or_more_ws_or_comment(p)
        p, name = self.var_name(p)

        def eqs(q):
            q = self.zero_or_more_ws_or_comment(q)
            return self.tag_any(q, ("=", ":="))

        p = self.cut(eqs, p)
        return p, name

    def assignment(self, p):
        p, name = self.let_assignment_expr(p)
        try:
            q, v = self.parse_value(p)
            return q, {"var": name, "value": ("Value", P.from_value(_lit(v)))}
        except Err:
            pass
        try:
            q = self.zero_or_more_ws_or_comment(p)
            q, f = self.function_expr(q)
            return q, {"var": name, "value": ("Func", f)}
        except (Err, Fail):
            pass

        def acc(q):
            q = self.zero_or_more_ws_or_comment(q)
            return self.access(q)

        q, a = self.cut(acc, p)
        return q, {"var": name, "value": ("Access", a)}

    def when(self, p):
        return self.tag_any(p, ("when", "WHEN"))

    def when_conditions(self, p, cond):
        p = self.zero_or_more_ws_or_comment(p)
        p = self.when(p)

        def rest(q):
            q = self.one_or_more_ws_or_comment(q)
            return cond(q)

        return self.cut(rest, p)

    def block(self, p, clause_parser):
        p = self.white_space(p, "{")
        assigns, conj = [], []

        def item(q):
            try:
                r = self.zero_or_more_ws_or_comment(q)
                r, a = self.assignment(r)
                return r, ("let", a)
            except Err:
                pass
            r, d = self.disjunction_clauses(q, clause_parser)
            return r, ("conj", d)

        try:
            p, v = item(p)
        except Err:
            raise Err(p)   # fold_many1
        items = [v]
        while True:
            try:
                q, v = item(p)
            except Err:
                break
            items.append(v)
            p = q
        for k, v in items:
            (assigns if k == "let" else conj).append(v)
        p = self.cut(lambda q: self.white_space(q, "}"), p)
        return p, (assigns, conj)

    def type_name(self, p):
        try:
            q, a = self.var_name(p)
            q = self.tag(q, "::")
            q, b = self.var_name(q)
            q = self.tag(q, "::")
            q, c = self.var_name(q)
            if self.s.startswith("::MODULE", q):
                q += len("::MODULE")
            return q, "%s::%s::%s" % (a, b, c)
        except Err:
            pass
        q, a = self.var_name(p)
        q = self.tag(q, "::")
        q, b = self.var_name(q)
        return q, "%s::%s" % (a, b)

    def type_block(self, p):
        location = self.loc(p)
        p, name = self.type_name(p)
        p = self.cut(self.one_or_more_ws_or_comment, p)
        conditions = None
        try:
            p, conditions = self.when_conditions(p, self.single_clauses)
        except Err:
            pass
        if conditions is not None:
            p, (assigns, conj) = self.cut(self.block, p, self.clause)
        else:
            try:
                p, (assigns, conj) = self.block(p, self.clause)
            except Err:
                def one(q):
                    q = self.zero_or_more_ws_or_comment(q)
                    return self.clause(q)
                p, c = self.cut(one, p)
                assigns, conj = [], [[c]]
        type_clause = {"kind": "Clause", "query": {"query": [("Key", "Type")], "match_all": True},
                       "comparator": ("Eq", False),
                       "compare_with": ("Value", P.PV(P.STRING, "", 0, 0, name)),
                       "custom_message": None, "location": location, "negation": False}
        return p, {"type_name": name, "conditions": conditions,
                   "block": {"assignments": assigns, "conjunctions": conj},
                   "query": [("Key", "Resources"), ("AllValues", None), ("Filter", None, [[type_clause]])]}

    def when_block(self, p, conds, block_fn, wrap=True):
        p = self.zero_or_more_ws_or_comment(p)
        p, c = self.when_conditions(p, conds)
        p, (assigns, conj) = self.block(p, block_fn)
        return p, {"kind": "WhenBlock", "conditions": c,
                   "block": {"assignments": assigns, "conjunctions": conj}}

    def rule_block_clause(self, p):
        try:
            q = self.zero_or_more_ws_or_comment(p)
            q, tb = self.type_block(q)
            return q, {"kind": "TypeBlock", "type_block": tb}
        except Err:
            pass
        try:
            q = self.zero_or_more_ws_or_comment(p)
            q, c = self.when_conditions(q, self.single_clauses)
            q, (assigns, conj) = self.block(q, self.clause_or_rule_clause)
            return q, {"kind": "WhenBlock", "conditions": c,
                       "block": {"assignments": assigns, "conjunctions": conj}}
        except Err:
            pass
        q = self.zero_or_more_ws_or_comment(p)
        q, c = self.clause_or_rule_clause(q)
        return q, {"kind": "GuardClause", "clause": c}

    def rule_block(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        p = self.tag(p, "rule")
        p = self.one_or_more_ws_or_comment(p)
        p, name = self.cut(self.var_name, p)
        conditions = None
        try:
            p, conditions = self.when_conditions(p, self.single_clauses)
        except Err:
            pass
        p, (assigns, conj) = self.cut(self.block, p, self.rule_block_clause)
        return p, {"rule_name": name, "conditions": conditions,
                   "block": {"assignments": assigns, "conjunctions": conj}}

    def parameter_names(self, p):
        p = self.char(p, "(")

        def elem(q):
            def inner(r):
                r = self.multispace0(r)
                r, v = self.var_name(r)
                return self.multispace0(r), v
            return self.cut(inner, q)

        p, names = self.separated_list1(p, lambda q: self.char(q, ","), elem)
        p = self.cut(self.char, p, ")")
        out = []
        for n in names:
            if n not in out:
                out.append(n)
        return p, out

    def parameterized_rule_block(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        p = self.tag(p, "rule")
        p = self.one_or_more_ws_or_comment(p)
        p, name = self.cut(self.var_name, p)
        p, params = self.parameter_names(p)
        p, (assigns, conj) = self.cut(self.block, p, self.rule_block_clause)
        return p, {"parameter_names": params,
                   "rule": {"rule_name": name, "conditions": None,
                            "block": {"assignments": assigns, "conjunctions": conj}}}

    def or_join(self, p):
        p = self.zero_or_more_ws_or_comment(p)
        p = self.tag_any(p, ("or", "OR", "|OR|"))
        return self.one_or_more_ws_or_comment(p)

    def rules_file(self):
        p = self.zero_or_more_ws_or_comment(0)
        if p >= self.n:
            return None
        exprs = []

        def one(q):
            q = self.zero_or_more_ws_or_comment(q)
            for kind, f in (("Assignment", self.assignment),
                            ("ParamRule", self.parameterized_rule_block),
                            ("Rule", self.rule_block),
                            ("DefaultTypeBlock", lambda r: self.disjunction_clauses(r, self.type_block)),
                            ("DefaultWhenBlock", lambda r: self.when_block(r, self.single_clauses,
                                                                           self.clause_or_rule_clause)),
                            ("DefaultClause", lambda r: self.disjunction_clauses(r, self.clause))):
                try:
                    r, v = f(q)
                    return self.zero_or_more_ws_or_comment(r), (kind, v)
                except Err:
                    if kind == "DefaultClause":
                        raise
                    continue

        try:
            p0 = p
            try:
                p, e = one(p)
            except Err:
                raise Err(p0)   # fold_many1: from_error_kind(input, Many1)
            exprs.append(e)
            while True:
                try:
                    q, e = one(p)
                except Err:
                    break
                exprs.append(e)
                p = q
            if p != self.n:
                raise Err(p)    # all_consuming: Eof
        except (Err, Fail) as e:
            raise GuardError("ParseError", "Parsing Error " + self.error_text(e.pos, e.ctx))

        assignments, named, param, default = [], [], [], []
        for kind, v in exprs:
            if kind == "Rule":
                named.append(v)
            elif kind == "ParamRule":
                param.append(v)
            elif kind == "Assignment":
                assignments.append(v)
            elif kind == "DefaultClause":
                default.append([{"kind": "GuardClause", "clause": c} for c in v])
            elif kind == "DefaultTypeBlock":
                default.append([{"kind": "TypeBlock", "type_block": t} for t in v])
            elif kind == "DefaultWhenBlock":
                default.append([{"kind": "WhenBlock", "conditions": v["conditions"], "block": v["block"]}])
        if default:
            name = "default" if self.file.strip() == "" else "%s/default" % self.file
            named.insert(0, {"rule_name": name, "conditions": None,
                             "block": {"assignments": [], "conjunctions": default}})
        return {"assignments": assignments, "guard_rules": named, "parameterized_rules": param}


UNARY_OPS = {"Exists", "Empty", "IsString", "IsList", "IsMap", "IsBool", "IsInt", "IsFloat", "IsNull"}


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def _is_variable(part):
    return part[0] == "Key" and part[1].startswith("%")


def _lit(v):
    """parser literal -> pv.from_value payload form"""
    kind, payload = v
    if kind == "List":
        return (P.LIST, [_lit(e) for e in payload])
    if kind == "Map":
        return (P.MAP, [(k, _lit(e)) for k, e in payload])
    return ({"Null": P.NULL, "String": P.STRING, "Regex": P.REGEX, "Bool": P.BOOL, "Int": P.INT,
             "Float": P.FLOAT, "Char": P.CHAR, "RangeInt": P.RANGE_INT, "RangeFloat": P.RANGE_FLOAT,
             "RangeChar": P.RANGE_CHAR}[kind], payload)


def parse_rules(text: str, file_name: str):
    """``rules_file`` parser.rs:1840-1932.  Returns None for an empty/comment-only file."""
    return Parser(text, file_name).rules_file()


# ---------------------------------------------------------------------------
# Display of AST pieces (context strings), exprs.rs:286-393
# ---------------------------------------------------------------------------
CMP_DISPLAY = {
    "Eq": "EQUALS", "In": "IN", "Gt": "GREATER THAN", "Lt": "LESS THAN", "Ge": "GREATER THAN EQUALS",
    "Le": "LESS THAN EQUALS", "Exists": "EXISTS", "Empty": "EMPTY", "IsString": "IS STRING",
    "IsBool": "IS BOOL", "IsInt": "IS INT", "IsList": "IS LIST", "IsMap": "IS MAP", "IsNull": "IS NULL",
    "IsFloat": "IS FLOAT",
}


def part_display(part):
    k = part[0]
    if k == "Key":
        return part[1]
    if k == "AllIndices":
        return "[*]"
    if k == "AllValues":
        return "*"
    if k == "Index":
        return str(part[1])
    if k == "Filter":
        return "%s (filter-clauses)" % (part[1] or "")
    if k == "MapKeyFilter":
        return "%s (map-key-filter-clauses)" % (part[1] or "")
    return "_"


def slice_display(parts, item_display=part_display):
    q = ""
    first = True
    for it in parts:
        if not first:
            q = "%s.%s" % (q, item_display(it))
        else:
            q = item_display(it)
        first = False
    return q.replace(".[", "[")


def let_value_display(lv):
    k = lv[0]
    if k == "Access":
        return slice_display(lv[1]["query"])
    if k == "Value":
        return P.value_only(lv[1])
    f = lv[1]
    return "%s(%s)" % (f["name"], ", ".join(let_value_display(x) for x in f["parameters"]))


def display_comparator(cmp):
    op, neg = cmp
    return "%s%s " % ("not " if neg else "", CMP_DISPLAY[op])


def gac_display(c):
    ac = "%s %s %s" % (slice_display(c["query"]["query"]), display_comparator(c["comparator"]),
                       let_value_display(c["compare_with"]) if c["compare_with"] is not None else "")
    return "%s %s" % ("not" if c["negation"] else "", ac)


def file_location_display(loc):
    return "Location[file:%s, line:%d, column:%d]" % (loc["file"], loc["line"], loc["column"])


def named_rule_display(c):
    return "Rule(%s@%s)" % (c["dependent_rule"], file_location_display(c["location"]))
