"""Evaluator restatement (TEST INFRASTRUCTURE ONLY -- the parity oracle).

Restates, function for function:
  * ``guard/src/rules/eval.rs``            (clause / block / rule / file evaluation)
  * ``guard/src/rules/eval/operators.rs``  (==, IN, <, >, <=, >= and ``not`` reverse diffs)
  * ``guard/src/rules/eval_context.rs:32-1606`` (query engine, scopes, record tracker)
  * ``guard/src/rules/functions/collections.rs`` (``count``)

Query results are tuples: ``('L', pv)`` Literal, ``('R', pv)`` Resolved,
``('U', UnResolved)``.  Records are ``Event`` objects (``EventRecord``).
"""
from .errors import GuardError
from . import pv as P
from .parser import slice_display, gac_display, named_rule_display, file_location_display, UNARY_OPS
from . import cruet

PASS, FAIL, SKIP = "PASS", "FAIL", "SKIP"


def status_and(a, b):
    """Status::and rules/mod.rs:122-133"""
    if a == FAIL:
        return FAIL
    if a == PASS:
        return FAIL if b == FAIL else PASS
    return b


class UnResolved:
    __slots__ = ("traversed_to", "remaining_query", "reason")

    def __init__(self, traversed_to, remaining_query, reason):
        self.traversed_to = traversed_to
        self.remaining_query = remaining_query
        self.reason = reason


def qr_debug(q):
    k, v = q
    if k == "L":
        return "Literal(%s)" % P.rust_debug(v)
    if k == "R":
        return "Resolved(%s)" % P.rust_debug(v)
    return "UnResolved(UnResolved { traversed_to: %s, remaining_query: %s, reason: %s })" % (
        P.rust_debug(v.traversed_to), P.rust_debug_str(v.remaining_query),
        "None" if v.reason is None else "Some(%s)" % P.rust_debug_str(v.reason))


class Event:
    __slots__ = ("context", "container", "children")

    def __init__(self, context):
        self.context = context
        self.container = None
        self.children = []


class RecordTracker:
    """eval_context.rs:999-1060"""

    def __init__(self):
        self.events = []
        self.final_event = None

    def start_record(self, context):
        self.events.append(Event(context))

    def end_record(self, context, record):
        if not self.events:
            raise GuardError("IncompatibleError",
                             "Event Record end with context %s did not have a corresponding start" % context)
        ev = self.events.pop()
        if ev.context != context:
            raise GuardError("IncompatibleError", "Event Record context start and end does not match %s" % context)
        ev.container = record
        if self.events:
            self.events[-1].children.append(ev)
        else:
            self.final_event = ev


# ---------------------------------------------------------------------------
# scopes (eval_context.rs:32-117, 1062-1606; eval.rs:1504-1572)
# ---------------------------------------------------------------------------
def _extract_variables(assignments):
    literals, queries, functions = {}, {}, {}
    for a in assignments:
        k, v = a["value"]
        if k == "Value":
            literals[a["var"]] = v
        elif k == "Access":
            queries[a["var"]] = v
        else:
            functions[a["var"]] = v
    return literals, queries, functions


class Scope:
    def __init__(self, root, assignments):
        self.root_value = root
        self.literals, self.variable_queries, self.function_expressions = _extract_variables(assignments)
        self.resolved_variables = {}


class RootScope:
    def __init__(self, rules_file, root):
        self.scope = Scope(root, rules_file["assignments"])
        self.rules = {}
        for r in rules_file["guard_rules"]:
            self.rules.setdefault(r["rule_name"], []).append(r)
        self.parameterized_rules = {}
        for pr in rules_file["parameterized_rules"]:
            self.parameterized_rules[pr["rule"]["rule_name"]] = pr
        self.rules_status = {}
        self.recorder = RecordTracker()

    def query(self, query):
        return query_retrieval(0, query, self.root(), self, None)

    def find_parameterized_rule(self, name):
        if name in self.parameterized_rules:
            return self.parameterized_rules[name]
        raise GuardError("MissingValue", "Parameterized Rule with name %s was not found, candidate [%s]" % (
            name, ", ".join(P.rust_debug_str(k) for k in self.parameterized_rules)))

    def root(self):
        return self.scope.root_value

    def rule_status(self, name):
        if name in self.rules_status:
            return self.rules_status[name]
        rules = self.rules.get(name)
        if rules is None:
            raise GuardError("MissingValue", "Rule %s by that name does not exist, Rule Names = [%s]" % (
                name, ", ".join(P.rust_debug_str(k) for k in self.rules)))
        status = SKIP
        for r in rules:
            s = eval_rule(r, self)
            if s != SKIP:
                status = s
                break
        self.rules_status[name] = status
        return status

    def resolve_variable(self, name):
        sc = self.scope
        if name in sc.literals:
            return [("L", sc.literals[name])]
        if name in sc.resolved_variables:
            return list(sc.resolved_variables[name])
        if name in sc.function_expressions:
            f = sc.function_expressions[name]
            res = resolve_function(f["name"], f["parameters"], self)
            sc.resolved_variables[name] = list(res)
            return res
        q = sc.variable_queries.get(name)
        if q is None:
            raise GuardError("MissingValue", "Could not resolve variable by name %s across scopes" % name)
        res = query_retrieval(0, q["query"], self.root(), self, None)
        if not q["match_all"]:
            res = [r for r in res if r[0] == "R"]
        sc.resolved_variables[name] = list(res)
        return res

    def add_variable_capture_key(self, name, key):
        self.scope.resolved_variables.setdefault(name, []).append(("R", key))

    def start_record(self, c):
        self.recorder.start_record(c)

    def end_record(self, c, r):
        self.recorder.end_record(c, r)


class BlockScope:
    def __init__(self, block, root, parent):
        self.scope = Scope(root, block["assignments"])
        self.parent = parent

    def query(self, query):
        return query_retrieval(0, query, self.root(), self, None)

    def find_parameterized_rule(self, name):
        return self.parent.find_parameterized_rule(name)

    def root(self):
        return self.scope.root_value

    def rule_status(self, name):
        return self.parent.rule_status(name)

    def resolve_variable(self, name):
        sc = self.scope
        if name in sc.literals:
            return [("L", sc.literals[name])]
        if name in sc.resolved_variables:
            return list(sc.resolved_variables[name])
        if name in sc.function_expressions:
            f = sc.function_expressions[name]
            res = resolve_function(f["name"], f["parameters"], self)
            sc.resolved_variables[name] = list(res)
            return res
        q = sc.variable_queries.get(name)
        if q is None:
            return self.parent.resolve_variable(name)
        res = query_retrieval(0, q["query"], self.root(), self, None)
        if not q["match_all"]:
            res = [r for r in res if r[0] == "R"]
        sc.resolved_variables[name] = list(res)
        return res

    def add_variable_capture_key(self, name, key):
        self.parent.add_variable_capture_key(name, key)

    def start_record(self, c):
        self.parent.start_record(c)

    def end_record(self, c, r):
        self.parent.end_record(c, r)


class ValueScope:
    def __init__(self, root, parent):
        self.root_value = root
        self.parent = parent

    def query(self, query):
        return query_retrieval(0, query, self.root(), self.parent, None)

    def find_parameterized_rule(self, name):
        return self.parent.find_parameterized_rule(name)

    def root(self):
        return self.root_value

    def rule_status(self, name):
        return self.parent.rule_status(name)

    def resolve_variable(self, name):
        return self.parent.resolve_variable(name)

    def add_variable_capture_key(self, name, key):
        self.parent.add_variable_capture_key(name, key)

    def start_record(self, c):
        self.parent.start_record(c)

    def end_record(self, c, r):
        self.parent.end_record(c, r)


class ResolvedParameterContext:
    def __init__(self, call_rule, resolved, parent):
        self.call_rule = call_rule
        self.resolved_parameters = resolved
        self.parent = parent

    def query(self, query):
        return self.parent.query(query)

    def find_parameterized_rule(self, name):
        return self.parent.find_parameterized_rule(name)

    def root(self):
        return self.parent.root()

    def rule_status(self, name):
        return self.parent.rule_status(name)

    def resolve_variable(self, name):
        if name in self.resolved_parameters:
            return list(self.resolved_parameters[name])
        return self.parent.resolve_variable(name)

    def add_variable_capture_key(self, name, key):
        self.parent.add_variable_capture_key(name, key)

    def start_record(self, c):
        self.parent.start_record(c)

    def end_record(self, c, r):
        if r[0] == "RuleCheck" and r[1] == self.call_rule["named_rule"]["dependent_rule"]:
            r = ("RuleCheck", r[1], r[2], self.call_rule["named_rule"]["custom_message"])
        self.parent.end_record(c, r)


# ---------------------------------------------------------------------------
# functions  (eval_context.rs:2437-2472; functions/collections.rs)
# ---------------------------------------------------------------------------
def resolve_function(name, parameters, resolver):
    args = []
    for p in parameters:
        k, v = p
        if k == "Value":
            args.append([("L", v)])
        elif k == "Access":
            args.append(resolver.query(v["query"]))
        else:
            args.append(resolve_function(v["name"], v["parameters"], resolver))
    if name == "count":
        a = args[0]
        n = sum(1 for q in a if q[0] != "U")
        if not a:
            return [("R", P.PV(P.INT, "", 0, 0, 0))]
        first = a[0]
        src = first[1].traversed_to if first[0] == "U" else first[1]
        return [("R", P.PV(P.INT, src.path, src.line, src.col, n))]
    raise GuardError("Unsupported", "function %s() is outside the oracle's scope" % name)


# ---------------------------------------------------------------------------
# query engine  (eval_context.rs:118-924)
# ---------------------------------------------------------------------------
def _unresolved(current, reason, query_slice):
    return ("U", UnResolved(current, slice_display(query_slice), reason))


def retrieve_index(parent, index, elements, query):
    check = index if index >= 0 else -index
    if check < len(elements):
        return ("R", elements[check])
    return _unresolved(parent, "Array Index out of bounds for path = %s on index = %d inside Array = [%s], remaining query = %s"
                       % (parent.path_display(), index, ", ".join(P.rust_debug(e) for e in elements),
                          slice_display(query)), query)


def accumulate(parent, query_index, query, elements, resolver, converter):
    if not elements:
        return [_unresolved(parent, "No more entries for value at path = %s on type = %s "
                            % (parent.path_display(), parent.type_info()), query[query_index:])]
    out = []
    for e in elements:
        out.extend(query_retrieval(query_index + 1, query, e, resolver, converter))
    return out


def accumulate_map(parent, mv, query_index, query, resolver, converter, func):
    if not mv.values:
        return [_unresolved(parent, "No more entries for value at path = %s on type = %s "
                            % (parent.path_display(), parent.type_info()), query[query_index:])]
    out = []
    for key, each in zip(mv.keys, mv.values.values()):
        vr = ValueScope(each, resolver)
        out.extend(func(query_index + 1, query, key, each, vr, converter))
    return out


def check_and_delegate(conjunctions, name):
    def f(index, query, key, value, ctx, converter):
        context = "Filter/Map#%d" % len(conjunctions)
        ctx.start_record(context)
        try:
            status = eval_conjunction_clauses(conjunctions, ctx, eval_guard_clause)
        except GuardError:
            ctx.end_record(context, ("Filter", FAIL))
            raise
        ctx.end_record(context, ("Filter", status))
        if name is not None and status == PASS:
            ctx.add_variable_capture_key(name, key)
        if status == PASS:
            return query_retrieval(index, query, value, ctx, converter)
        return []
    return f


def query_retrieval(query_index, query, current, resolver, converter):
    if query_index >= len(query):
        return [("R", current)]
    part = query[query_index]
    if query_index == 0 and part[0] == "Key" and part[1].startswith("%"):
        retrieved = resolver.resolve_variable(part[1][1:])
        out = []
        for each in retrieved:
            if each[0] == "U":
                out.append(each)
                continue
            value = each[1]
            if query_index + 1 < len(query):
                index = query_index + 2 if query[query_index + 1][0] == "AllIndices" else query_index + 1
            else:
                index = query_index + 1
            if index < len(query):
                scope = ValueScope(value, resolver)
                out.extend(query_retrieval(index, query, value, scope, converter))
            else:
                out.append(each)
        return out

    k = part[0]
    if k == "This":
        return query_retrieval(query_index + 1, query, current, resolver, converter)

    if k == "Key":
        key = part[1]
        idx = _parse_i32(key)
        if idx is not None:
            if current.kind == P.LIST:
                r = retrieve_index(current, idx, current.val, query)
                if r[0] == "R":
                    return query_retrieval(query_index + 1, query, r[1], resolver, converter)
                return [r]
            return [("U", UnResolved(current, slice_display(query),
                                     "Attempting to retrieve from index %d but type is not an array at path %s"
                                     % (idx, current.path_display())))]
        if current.kind == P.MAP:
            mv = current.val
            path_disp = current.path_display()
            if key.startswith("%"):
                var = key[1:]
                keys = resolver.resolve_variable(var)
                if len(query) > query_index + 1:
                    nxt = query[query_index + 1]
                    if nxt[0] in ("AllIndices", "Key"):
                        pass
                    elif nxt[0] == "Index":
                        check = nxt[1] if nxt[1] >= 0 else -nxt[1]
                        if check < len(keys):
                            keys = [keys[check]]
                        else:
                            return [_unresolved(current, "Index %d on the set of values returned for variable %s on the join, is out of bounds. Length %d, Values = [%s]"
                                                % (check, var, len(keys), ", ".join(qr_debug(q) for q in keys)),
                                                query[query_index:])]
                    else:
                        raise GuardError("IncompatibleError", "This type of query %s based variable interpolation is not supported %s, %s"
                                         % (_part_disp(query[1]), current.type_info(), slice_display(query)))
                acc = []
                for each_key in keys:
                    if each_key[0] == "U":
                        ur = each_key[1]
                        acc.append(_unresolved(current, "Keys returned for variable %s could not completely resolve. Path traversed until %s%s"
                                               % (var, ur.traversed_to.path_display(), ur.reason or ""),
                                               query[query_index:]))
                        continue
                    kv = each_key[1]
                    if kv.kind == P.STRING:
                        nxt = mv.values.get(kv.val)
                        if nxt is not None:
                            acc.extend(query_retrieval(query_index + 1, query, nxt, resolver, converter))
                        else:
                            acc.append(_unresolved(current, "Could not locate key = %s inside struct at path = %s"
                                                   % (kv.val, path_disp), query[query_index:]))
                    elif kv.kind == P.LIST:
                        for inner in kv.val:
                            if inner.kind == P.STRING:
                                nxt = mv.values.get(inner.val)
                                if nxt is not None:
                                    acc.extend(query_retrieval(query_index + 1, query, nxt, resolver, converter))
                                else:
                                    acc.append(_unresolved(current, "Could not locate key = %s inside struct at path = %s"
                                                           % (inner.val, inner.path_display()), query[query_index:]))
                            else:
                                raise GuardError("NotComparable", "Variable projections inside Query %s, is returning a non-string value for key %s, %s"
                                                 % (slice_display(query), kv.type_info(), _self_value_debug(kv)))
                    else:
                        raise GuardError("NotComparable", "Variable projections inside Query %s, is returning a non-string value for key %s, %s"
                                         % (slice_display(query), kv.type_info(), _self_value_debug(kv)))
                return acc
            val = mv.values.get(key)
            if val is not None:
                return query_retrieval(query_index + 1, query, val, resolver, converter)
            if converter is not None:
                conv = converter(key)
                val = mv.values.get(conv)
                if val is not None:
                    return query_retrieval(query_index + 1, query, val, resolver, converter)
            else:
                for cv in cruet.CONVERTERS:
                    val = mv.values.get(cv(key))
                    if val is not None:
                        return query_retrieval(query_index + 1, query, val, resolver, cv)
            return [_unresolved(current, "Could not find key %s inside struct at path %s" % (key, path_disp),
                                query[query_index:])]
        return [_unresolved(current, "Attempting to retrieve from key %s but type is not an struct type at path %s, Type = %s, Value = %s"
                            % (key, current.path_display(), current.type_info(), P.rust_debug(current)),
                            query[query_index:])]

    if k == "Index":
        index = part[1]
        if current.kind == P.LIST:
            r = retrieve_index(current, index, current.val, query)
            if r[0] == "R":
                return query_retrieval(query_index + 1, query, r[1], resolver, converter)
            return [r]
        return [_unresolved(current, "Attempting to retrieve from index %d but type is not an array at path %s, type %s"
                            % (index, current.path_display(), current.type_info()), query[query_index:])]

    if k == "AllIndices":
        name = part[1]
        if current.kind == P.LIST:
            return accumulate(current, query_index, query, current.val, resolver, converter)
        if current.kind == P.MAP:
            if name is None:
                return query_retrieval(query_index + 1, query, current, resolver, converter)

            def cap(index, q, key, value, ctx, conv):
                ctx.add_variable_capture_key(name, key)
                return query_retrieval(index, q, value, ctx, conv)
            return accumulate_map(current, current.val, query_index, query, resolver, converter, cap)
        return query_retrieval(query_index + 1, query, current, resolver, converter)

    if k == "AllValues":
        name = part[1]
        if current.kind == P.LIST:
            return accumulate(current, query_index, query, current.val, resolver, converter)
        if current.kind == P.MAP:
            def allv(index, q, key, value, ctx, conv):
                if name is not None:
                    ctx.add_variable_capture_key(name, key)
                return query_retrieval(index, q, value, ctx, conv)
            return accumulate_map(current, current.val, query_index, query, resolver, converter, allv)
        return query_retrieval(query_index + 1, query, current, resolver, converter)

    if k == "Filter":
        name, conjunctions = part[1], part[2]
        if current.kind == P.MAP:
            prev = query[query_index - 1][0]
            if prev in ("AllValues", "AllIndices"):
                return check_and_delegate(conjunctions, None)(query_index + 1, query, current, current, resolver, converter)
            if prev == "Key":
                if current.val.values:
                    return accumulate_map(current, current.val, query_index, query, resolver, converter,
                                          check_and_delegate(conjunctions, name))
                return []
            # `_ => unreachable!()` (eval_context.rs:752): a panic, ffi-support code -1 with its payload
            raise GuardError("Panic", "internal error: entered unreachable code")
        if current.kind == P.LIST:
            selected = []
            for each in current.val:
                context = "Filter/List#%d" % len(conjunctions)
                resolver.start_record(context)
                vr = ValueScope(each, resolver)
                try:
                    status = eval_conjunction_clauses(conjunctions, vr, eval_guard_clause)
                except GuardError:
                    resolver.end_record(context, ("Filter", FAIL))
                    raise
                resolver.end_record(context, ("Filter", status))
                if status == PASS:
                    selected.extend(query_retrieval(query_index + 1, query, each, resolver, converter))
            return selected
        if query[query_index - 1][0] == "AllIndices":
            vr = ValueScope(current, resolver)
            status = eval_conjunction_clauses(conjunctions, vr, eval_guard_clause)
            if status == PASS:
                return query_retrieval(query_index + 1, query, current, resolver, converter)
            return []
        return [_unresolved(current, "Filter on value type that was not a struct or array %s %s"
                            % (current.type_info(), current.path_display()), query[query_index:])]

    if k == "MapKeyFilter":
        clause = part[2]
        if current.kind == P.MAP:
            mv = current.val
            cw = clause["compare_with"]
            if cw[0] == "Access":
                rhs = query_retrieval(0, cw[1]["query"], current, resolver, converter)
            elif cw[0] == "Value":
                rhs = [("L", cw[1])]
            else:
                rhs = resolve_function(cw[1]["name"], cw[1]["parameters"], resolver)
            lhs = [("R", k2) for k2 in mv.keys]
            results = real_binary_operation(lhs, rhs, clause["comparator"], "", None, resolver)
            selected = []
            for q, st in results[1]:
                if q[0] == "R" and st == PASS:
                    if q[1].kind == P.STRING:
                        selected.append(("R", mv.values[q[1].val]))
                elif q[0] == "U":
                    selected.append(q)
            out = []
            for s in selected:
                if s[0] == "U":
                    out.append(s)
                else:
                    out.extend(query_retrieval(query_index + 1, query, s[1], resolver, converter))
            return out
        return [_unresolved(current, "Map Filter for keys was not a struct %s %s"
                            % (current.type_info(), current.path_display()), query[query_index:])]
    raise GuardError("Unsupported", "unknown query part %r" % (part,))


def _part_disp(part):
    from .parser import part_display
    return part_display(part)


def _self_value_debug(v):
    return "(%s, %s)" % (P._debug_path(v), P.rust_debug(v))


def _parse_i32(s):
    import re
    if not re.match(r"^[+-]?[0-9]+$", s):
        return None
    v = int(s)
    if v < -(1 << 31) or v >= (1 << 31):
        return None
    return v


# ---------------------------------------------------------------------------
# unary  (eval.rs:10-405)
# ---------------------------------------------------------------------------
def _element_empty(q):
    k, v = q
    if k == "U":
        return True
    if v.kind == P.LIST:
        return len(v.val) == 0
    if v.kind == P.MAP:
        return len(v.val.values) == 0
    if v.kind == P.STRING:
        return len(v.val) == 0
    if v.kind == P.BOOL:
        return False
    raise GuardError("IncompatibleError", "Attempting EMPTY operation on type %s that does not support it at %s"
                     % (v.type_info(), v.path_display()))


_IS_TYPE = {"IsString": P.STRING, "IsList": P.LIST, "IsMap": P.MAP, "IsInt": P.INT, "IsFloat": P.FLOAT,
            "IsBool": P.BOOL, "IsNull": P.NULL}


def _unary_fn(op):
    if op == "Exists":
        return lambda q: q[0] != "U"
    if op == "Empty":
        return _element_empty
    t = _IS_TYPE[op]
    return lambda q: q[0] != "U" and q[1].kind == t


def unary_operation(lhs_query, cmp, inverse, context, custom_message, ctx):
    lhs = ctx.query(lhs_query)
    last = lhs_query[-1]
    empty_on_expr = last[0] in ("Filter", "MapKeyFilter") or (
        last[0] == "Key" and last[1].startswith("%") and len(lhs_query) == 1)
    if empty_on_expr and cmp[0] == "Empty":
        if lhs:
            results = []
            for each in lhs:
                ctx.start_record(context)
                if each[0] in ("L", "R"):
                    res = each[1]
                    st = (not res.is_null()) if cmp[1] else res.is_null()
                    result = ("R", res)
                    status = PASS if st else FAIL
                else:
                    result = each
                    status = FAIL if cmp[1] else PASS
                if inverse:
                    status = FAIL if status == PASS else PASS
                if status == PASS:
                    ctx.end_record(context, ("ClauseValueCheck", ("Success",)))
                else:
                    ctx.end_record(context, ("ClauseValueCheck", ("Unary", {
                        "comparison": cmp, "from": result, "message": None,
                        "custom_message": custom_message})))
                results.append((result, status))
            return ("values", results)
        result = not cmp[1]
        if inverse:
            result = not result
        ctx.start_record(context)
        if result:
            ctx.end_record(context, ("ClauseValueCheck", ("Success",)))
            return ("empty", PASS)
        ctx.end_record(context, ("ClauseValueCheck", ("NoValueForEmptyCheck", custom_message)))
        return ("empty", FAIL)

    if not lhs:
        return ("empty", SKIP)

    base = _unary_fn(cmp[0])
    results = []
    for each in lhs:
        ctx.start_record(context)
        try:
            r = base(each)
            if cmp[1]:
                r = not r
            if inverse:
                r = not r
        except GuardError as e:
            ctx.end_record(context, ("ClauseValueCheck", ("Unary", {
                "comparison": cmp, "from": each, "message": e.display(), "custom_message": custom_message})))
            raise
        if not r:
            ctx.end_record(context, ("ClauseValueCheck", ("Unary", {
                "comparison": cmp, "from": each, "message": None, "custom_message": custom_message})))
        else:
            ctx.end_record(context, ("ClauseValueCheck", ("Success",)))
        results.append((each, PASS if r else FAIL))
    return ("values", results)


# ---------------------------------------------------------------------------
# operators.rs
# ---------------------------------------------------------------------------
def _selected(results, on_unresolved):
    out = []
    for q in results:
        if q[0] == "U":
            on_unresolved(q[1])
        else:
            out.append(q[1])
    return out


def _flattened(results, on_unresolved):
    out = []
    for q in results:
        if q[0] == "U":
            on_unresolved(q[1])
        else:
            v = q[1]
            if v.kind == P.LIST:
                out.extend(v.val)
            else:
                out.append(v)
    return out


# ValueEvalResult representation:
#   ('LhsUnresolved', ur)
#   ('RhsUnresolved', ur, lhs)
#   ('NotComparable', reason, lhs, rhs)
#   ('Success'|'Fail', compare) where compare is
#        ('Value', lhs, rhs) | ('ValueIn', lhs, rhs) | ('ListIn', diff, lhs, rhs) | ('QueryIn', diff, lhs[], rhs[])

def _match_value(l, r, comparator):
    try:
        ok = comparator(l, r)
    except P.NotComparable as e:
        return ("NotComparable", e.msg, l, r)
    return ("Success" if ok else "Fail", ("Value", l, r))


def _contains(lst, v):
    return any(P.pv_eq(x, v) for x in lst)


def _string_in(l, r):
    if l.kind == P.STRING and r.kind == P.STRING:
        return ("Success" if l.val in r.val else "Fail", ("Value", l, r))
    return ("NotComparable", "Type not comparable, %s, %s" % (P.display(l), P.display(r)), l, r)


def _contained_in(l, r):
    if l.kind == P.LIST:
        if r.kind == P.LIST:
            rl = r.val
            if rl and rl[0].is_list():
                if _contains(rl, l):
                    return ("Success", ("ListIn", [], l, r))
                return ("Fail", ("ListIn", [l], l, r))
            diff = [e for e in l.val if not _contains(rl, e)]
            return ("Success" if not diff else "Fail", ("ListIn", diff, l, r))
        return ("NotComparable", "Can not compare type %s, %s" % (P.display(l), P.display(r)), l, r)
    if r.kind == P.LIST:
        return ("Success" if _contains(r.val, l) else "Fail", ("ValueIn", l, r))
    return _match_value(l, r, P.compare_eq)


def _is_literal(results):
    if len(results) == 1 and results[0][0] == "L":
        return results[0][1]
    return None


def _common_op(lhs, rhs, comparator):
    results = []
    lhs_flat = _flattened(lhs, lambda ur: results.append(("LhsUnresolved", ur)))
    rhs_flat = _flattened(rhs, lambda ur: results.extend(("RhsUnresolved", ur, l) for l in lhs_flat))
    for l in lhs_flat:
        for r in rhs_flat:
            results.append(_match_value(l, r, comparator))
    return results


def _in_op(lhs, rhs):
    results = []
    l, r = _is_literal(lhs), _is_literal(rhs)
    if l is not None and r is not None:
        res = _string_in(l, r)
        if res[0] != "Success":
            res = _contained_in(l, r)
        results.append(res)
    elif l is not None:
        rhs_sel = _selected(rhs, lambda ur: results.append(("RhsUnresolved", ur, l)))
        if any(e.is_list() for e in rhs_sel):
            for e in rhs_sel:
                results.append(_contained_in(l, e))
        elif l.kind == P.LIST:
            diff = [e for e in l.val if not _contains(rhs_sel, e)]
            results.append(("Success" if not diff else "Fail", ("QueryIn", diff, [l], rhs_sel)))
        else:
            for e in rhs_sel:
                results.append(_contained_in(l, e))
    elif r is not None:
        lhs_sel = _selected(lhs, lambda ur: results.append(("LhsUnresolved", ur)))
        for lv in lhs_sel:
            if r.kind == P.STRING:
                if lv.kind == P.LIST:
                    for e in lv.val:
                        results.append(_string_in(e, r))
                else:
                    results.append(_string_in(lv, r))
            else:
                results.append(_contained_in(lv, r))
    else:
        lhs_sel = _selected(lhs, lambda ur: results.append(("LhsUnresolved", ur)))
        rhs_sel = _selected(rhs, lambda ur: results.extend(("RhsUnresolved", ur, x) for x in lhs_sel))
        diff = []
        for el in lhs_sel:
            for er in rhs_sel:
                if _contained_in(el, er)[0] == "Success":
                    break
            else:
                diff.append(el)
        results.append(("Success" if not diff else "Fail", ("QueryIn", diff, lhs_sel, rhs_sel)))
    return results


def _eq_op(lhs, rhs):
    results = []
    l, r = _is_literal(lhs), _is_literal(rhs)
    if l is not None and r is not None:
        results.append(_match_value(l, r, P.compare_eq))
    elif l is not None:
        rhs_sel = _selected(rhs, lambda ur: results.append(("RhsUnresolved", ur, l)))
        if l.kind == P.LIST:
            for e in rhs_sel:
                results.append(_match_value(l, e, P.compare_eq))
        else:
            for er in rhs_sel:
                if er.kind == P.LIST:
                    for e in er.val:
                        results.append(_match_value(l, e, P.compare_eq))
                else:
                    results.append(_match_value(l, er, P.compare_eq))
    elif r is not None:
        lhs_sel = _selected(lhs, lambda ur: results.append(("LhsUnresolved", ur)))
        if r.kind == P.LIST:
            for e in lhs_sel:
                if e.is_scalar() and len(r.val) == 1:
                    results.append(_match_value(e, r.val[0], P.compare_eq))
                else:
                    results.append(_match_value(e, r, P.compare_eq))
        else:
            for e in lhs_sel:
                if e.kind == P.LIST:
                    for x in e.val:
                        results.append(_match_value(x, r, P.compare_eq))
                else:
                    results.append(_match_value(e, r, P.compare_eq))
    else:
        lhs_sel = _selected(lhs, lambda ur: results.append(("LhsUnresolved", ur)))
        rhs_sel = _selected(rhs, lambda ur: results.extend(("RhsUnresolved", ur, x) for x in lhs_sel))
        if len(lhs_sel) > len(rhs_sel):
            diff = [e for e in lhs_sel if not _contains(rhs_sel, e)]
        else:
            diff = [e for e in rhs_sel if not _contains(lhs_sel, e)]
        results.append(("Success" if not diff else "Fail", ("QueryIn", diff, lhs_sel, rhs_sel)))
    return results


_COMMON = {"Lt": P.compare_lt, "Gt": P.compare_gt, "Le": P.compare_le, "Ge": P.compare_ge}


def _reverse_diff(diff, other):
    return [e for e in other if not _contains(diff, e)]


def compare(cmp, lhs, rhs):
    """``impl Comparator for (CmpOperator, bool)`` operators.rs:648-787"""
    op, neg = cmp
    if not lhs or not rhs:
        return None  # Skip
    if op == "Eq":
        r = _eq_op(lhs, rhs)
    elif op == "In":
        r = _in_op(lhs, rhs)
    elif op in _COMMON:
        r = _common_op(lhs, rhs, _COMMON[op])
    else:
        raise GuardError("IncompatibleError", "Operation %s NOT PERMITTED" % op)
    if not neg:
        return r
    out = []
    for e in r:
        if e[0] == "Fail":
            c = e[1]
            if c[0] == "QueryIn":
                _, diff, ql, qr = c
                if len(rhs) >= len(lhs) and op == "Eq":
                    rd = _reverse_diff(diff, qr)
                else:
                    rd = _reverse_diff(diff, ql)
                out.append(("Success" if not rd else "Fail", ("QueryIn", rd, ql, qr)))
            elif c[0] == "ListIn":
                _, diff, ll, lr = c
                rd = [x for x in ll.val if not _contains(diff, x)]
                out.append(("Success" if not rd else "Fail", ("ListIn", rd, ll, lr)))
            else:
                out.append(("Success", c))
        elif e[0] == "Success":
            c = e[1]
            if c[0] == "QueryIn":
                out.append(("Fail", ("QueryIn", list(c[2]), c[2], c[3])))
            elif c[0] == "ListIn":
                out.append(("Fail", ("ListIn", list(c[2].val), c[2], c[3])))
            else:
                out.append(("Fail", c))
        else:
            out.append(e)
    return out


def _record_cmp_fail(ctx, context, custom_message, cmp, frm, to, message=None):
    ctx.start_record(context)
    ctx.end_record(context, ("ClauseValueCheck", ("Comparison", {
        "status": FAIL, "message": message, "custom_message": custom_message, "comparison": cmp,
        "from": frm, "to": to})))


def _record_in_fail(ctx, context, custom_message, cmp, frm, to):
    ctx.start_record(context)
    ctx.end_record(context, ("ClauseValueCheck", ("InComparison", {
        "status": FAIL, "message": None, "custom_message": custom_message, "comparison": cmp,
        "from": frm, "to": to})))


def _record_success(ctx, context):
    ctx.start_record(context)
    ctx.end_record(context, ("ClauseValueCheck", ("Success",)))


def binary_operation(lhs_query, rhs, cmp, context, custom_message, ctx):
    """eval.rs:765-974"""
    lhs = ctx.query(lhs_query)
    results = compare(cmp, lhs, rhs)
    if results is None:
        return ("empty", SKIP)
    statuses = []
    for e in results:
        k = e[0]
        if k == "LhsUnresolved":
            _record_cmp_fail(ctx, context, custom_message, cmp, ("U", e[1]), None)
            statuses.append((("U", e[1]), FAIL))
        elif k == "RhsUnresolved":
            _record_cmp_fail(ctx, context, custom_message, cmp, ("R", e[2]), ("U", e[1]))
            statuses.append((("R", e[2]), FAIL))
        elif k == "NotComparable":
            _record_cmp_fail(ctx, context, custom_message, cmp, ("R", e[2]), ("R", e[3]), message=e[1])
            statuses.append((("R", e[2]), FAIL))
        elif k == "Success":
            c = e[1]
            if c[0] == "ListIn":
                _record_success(ctx, context)
                statuses.append((("R", c[2]), PASS))
            elif c[0] == "QueryIn":
                for each in c[2]:
                    _record_success(ctx, context)
                    statuses.append((("R", each), PASS))
            else:
                _record_success(ctx, context)
                statuses.append((("R", c[1]), PASS))
        else:
            c = e[1]
            if c[0] == "Value":
                _record_cmp_fail(ctx, context, custom_message, cmp, ("R", c[1]), ("R", c[2]))
                statuses.append((("R", c[1]), FAIL))
            elif c[0] == "ValueIn":
                _record_in_fail(ctx, context, custom_message, cmp, ("R", c[1]), [("R", c[2])])
                statuses.append((("R", c[1]), FAIL))
            elif c[0] == "ListIn":
                _record_in_fail(ctx, context, custom_message, cmp, ("R", c[2]), [("R", c[3])])
                statuses.append((("R", c[2]), FAIL))
            else:
                rhs_all = [("R", x) for x in c[3]]
                for l in c[1]:
                    _record_in_fail(ctx, context, custom_message, cmp, ("R", l), list(rhs_all))
                    statuses.append((("R", l), FAIL))
    return ("values", statuses)


# real_binary_operation (eval.rs:976-1075), used by MapKeyFilter
def _each_lhs_compare(cmpf, lhs, rhs):
    out = []
    for r in rhs:
        if r[0] == "U":
            out.append(("UnResolvedRhs", r, lhs))
            continue
        rv = r[1]
        try:
            out.append(("Comparable", cmpf(lhs, rv), lhs, rv))
            continue
        except P.NotComparable as e:
            reason = e.msg
        if lhs.is_list():
            for each in lhs.val:
                try:
                    out.append(("Comparable", cmpf(each, rv), each, rv))
                except P.NotComparable as e2:
                    out.append(("NotComparable", e2.msg, each, rv))
            continue
        if lhs.is_scalar() and r[0] == "L" and rv.kind == P.LIST and len(rv.val) == 1:
            inner = rv.val[0]
            try:
                out.append(("Comparable", cmpf(lhs, inner), lhs, inner))
            except P.NotComparable as e2:
                out.append(("NotComparable", e2.msg, lhs, inner))
            continue
        out.append(("NotComparable", reason, lhs, rv))
    return out


def _in_cmp(not_in):
    def f(l, r):
        if l.kind == P.STRING and r.kind == P.STRING:
            res = l.val in r.val
            return (not res) if not_in else res
        if r.kind == P.LIST:
            found = False
            for e in r.val:
                if P.compare_eq(l, e):
                    found = True
            return (not found) if not_in else found
        res = P.compare_eq(l, r)
        return (not res) if not_in else res
    return f


def _not_compare(f, invert):
    return lambda l, r: (not f(l, r)) if invert else f(l, r)


def real_binary_operation(lhs, rhs, cmp, context, custom_message, ctx):
    statuses = []
    if cmp[0] == "Eq" and len(rhs) > 1:
        cmp = ("In", cmp[1])
    for each in lhs:
        if each[0] == "U":
            _record_cmp_fail(ctx, context, custom_message, cmp, each, None)
            statuses.append((each, FAIL))
            continue
        l = each[1]
        op, neg = cmp
        if op == "In":
            r = _each_lhs_compare(_in_cmp(neg), l, rhs)
        else:
            base = {"Eq": P.compare_eq, "Ge": P.compare_ge, "Gt": P.compare_gt, "Lt": P.compare_lt,
                    "Le": P.compare_le}[op]
            r = _each_lhs_compare(_not_compare(base, neg), l, rhs)
        if op == "In":
            # report_at_least_one: grouping by lhs value (HashMap order; deterministic for one lhs)
            groups = []
            for res in r:
                if res[0] == "UnResolvedRhs":
                    key, rq = res[2], res[1]
                else:
                    key, rq = res[2], ("R", res[3])
                for g in groups:
                    if P.pv_eq(g[0], key):
                        g[1].append((res, rq))
                        break
                else:
                    groups.append((key, [(res, rq)]))
            for key, items in groups:
                if any(x[0][0] == "Comparable" and x[0][1] for x in items):
                    _record_success(ctx, context)
                    statuses.append((("R", key), PASS))
                else:
                    _record_in_fail(ctx, context, custom_message, cmp, ("R", key), [x[1] for x in items])
                    statuses.append((("R", key), FAIL))
        else:
            for res in r:
                if res[0] == "Comparable":
                    ok, lv, rv = res[1], res[2], res[3]
                    frm, to = ("R", lv), ("R", rv)
                elif res[0] == "NotComparable":
                    ok, frm, to = False, ("R", res[2]), ("R", res[3])
                else:
                    ok, frm, to = False, ("R", res[2]), res[1]
                if ok:
                    _record_success(ctx, context)
                    statuses.append((frm, PASS))
                else:
                    _record_cmp_fail(ctx, context, custom_message, cmp, frm, to)
                    statuses.append((frm, FAIL))
    return ("values", statuses)


# ---------------------------------------------------------------------------
# clauses / blocks / rules  (eval.rs:1077-2065)
# ---------------------------------------------------------------------------
def eval_guard_access_clause(gac, ctx):
    all_ = gac["query"]["match_all"]
    blk_context = "GuardAccessClause#block%s" % gac_display(gac)
    ctx.start_record(blk_context)
    cmp = gac["comparator"]
    try:
        if cmp[0] in UNARY_OPS:
            res = unary_operation(gac["query"]["query"], cmp, gac["negation"], gac_display(gac),
                                  gac["custom_message"], ctx)
        else:
            cw = gac["compare_with"]
            if cw is None:
                raise GuardError("NotComparable",
                                 "GuardAccessClause %s, did not have a RHS for compare operation" % blk_context)
            if cw[0] == "Value":
                rhs = [("L", cw[1])]
            elif cw[0] == "Access":
                rhs = ctx.query(cw[1]["query"])
            else:
                rhs = resolve_function(cw[1]["name"], cw[1]["parameters"], ctx)
            # NOTE: the clause-level ``not`` (gac.negation) is not applied to binary
            # operators in the reference (eval.rs:1146-1153)
            res = binary_operation(gac["query"]["query"], rhs, cmp, gac_display(gac), gac["custom_message"], ctx)
    except GuardError:
        ctx.end_record(blk_context, ("GuardClauseBlockCheck", FAIL, not all_))
        raise
    if res[0] == "empty":
        ctx.end_record(blk_context, ("GuardClauseBlockCheck", res[1], all_))
        return res[1]
    fails = sum(1 for _, s in res[1] if s == FAIL)
    passes = sum(1 for _, s in res[1] if s == PASS)
    if all_:
        outcome = FAIL if fails > 0 else PASS
    else:
        outcome = PASS if passes > 0 else FAIL
    ctx.end_record(blk_context, ("GuardClauseBlockCheck", outcome, not all_))
    return outcome


def eval_guard_named_clause(gnc, ctx):
    context = named_rule_display(gnc)
    ctx.start_record(context)
    try:
        status = ctx.rule_status(gnc["dependent_rule"])
    except GuardError as e:
        ctx.end_record(context, ("ClauseValueCheck", ("DependentRule", {
            "rule": gnc["dependent_rule"], "custom_message": gnc["custom_message"]})))
        raise
    if status == PASS:
        status = FAIL if gnc["negation"] else PASS
    else:
        status = PASS if gnc["negation"] else FAIL
    if status == PASS:
        ctx.end_record(context, ("ClauseValueCheck", ("Success",)))
    else:
        ctx.end_record(context, ("ClauseValueCheck", ("DependentRule", {
            "rule": gnc["dependent_rule"], "custom_message": gnc["custom_message"]})))
    return status


def eval_general_block_clause(block, ctx, eval_fn):
    scope = BlockScope(block, ctx.root(), ctx)
    return eval_conjunction_clauses(block["conjunctions"], scope, eval_fn)


def eval_guard_block_clause(bc, ctx):
    context = "BlockGuardClause#%s" % file_location_display(bc["location"])
    match_all = bc["query"]["match_all"]
    ctx.start_record(context)
    try:
        values = ctx.query(bc["query"]["query"])
    except GuardError:
        ctx.end_record(context, ("BlockGuardCheck", FAIL, not match_all))
        raise
    if not values:
        status = FAIL if bc["not_empty"] else SKIP
        ctx.end_record(context, ("BlockGuardCheck", status, not match_all))
        return status
    fails = passes = 0
    for each in values:
        if each[0] == "U":
            fails += 1
            ur = each[1]
            gctx = "GuardBlockAccessClause#%s" % file_location_display(bc["location"])
            ctx.start_record(gctx)
            ctx.end_record(gctx, ("ClauseValueCheck", ("MissingBlockValue", {
                "from": each, "custom_message": None,
                "message": "Query %s did not resolve to correct value, reason %s" % (
                    slice_display(bc["query"]["query"]), ur.reason or "")})))
        else:
            vr = ValueScope(each[1], ctx)
            try:
                st = eval_general_block_clause(bc["block"], vr, eval_guard_clause)
            except GuardError:
                ctx.end_record(context, ("BlockGuardCheck", FAIL, not match_all))
                raise
            if st == PASS:
                passes += 1
            elif st == FAIL:
                fails += 1
    if match_all:
        status = FAIL if fails > 0 else (PASS if passes > 0 else SKIP)
    else:
        status = PASS if passes > 0 else (FAIL if fails > 0 else SKIP)
    ctx.end_record(context, ("BlockGuardCheck", status, not match_all))
    return status


def eval_when_condition_block(context, conditions, block, ctx):
    ctx.start_record(context)
    when_context = "%s/When" % context
    ctx.start_record(when_context)
    try:
        st = eval_conjunction_clauses(conditions, ctx, eval_when_clause)
    except GuardError:
        ctx.end_record(when_context, ("WhenCondition", FAIL))
        ctx.end_record(context, ("WhenCheck", FAIL))
        raise
    if st != PASS:
        ctx.end_record(when_context, ("WhenCondition", st))
        ctx.end_record(context, ("WhenCheck", SKIP))
        return SKIP
    ctx.end_record(when_context, ("WhenCondition", PASS))
    try:
        st = eval_general_block_clause(block, ctx, eval_guard_clause)
    except GuardError:
        ctx.end_record(context, ("WhenCheck", FAIL))
        raise
    ctx.end_record(context, ("WhenCheck", st))
    return st


def eval_parameterized_rule_call(call, ctx):
    pr = ctx.find_parameterized_rule(call["named_rule"]["dependent_rule"])
    if len(pr["parameter_names"]) != len(call["parameters"]):
        raise GuardError("IncompatibleError", "Arity mismatch for called parameter rule %s, expected %d, got %d"
                         % (call["named_rule"]["dependent_rule"], len(pr["parameter_names"]), len(call["parameters"])))
    resolved = {}
    for i, p in enumerate(call["parameters"]):
        k, v = p
        name = pr["parameter_names"][i]
        if k == "Value":
            resolved[name] = [("R", v)]
        elif k == "Access":
            resolved[name] = ctx.query(v["query"])
        else:
            resolved[name] = resolve_function(v["name"], v["parameters"], ctx)
    return eval_rule(pr["rule"], ResolvedParameterContext(call, resolved, ctx))


def eval_guard_clause(gc, ctx):
    k = gc["kind"]
    if k == "Clause":
        return eval_guard_access_clause(gc, ctx)
    if k == "NamedRule":
        return eval_guard_named_clause(gc, ctx)
    if k == "BlockClause":
        return eval_guard_block_clause(gc, ctx)
    if k == "WhenBlock":
        return eval_when_condition_block("GuardConditionClause", gc["conditions"], gc["block"], ctx)
    if k == "ParamRule":
        return eval_parameterized_rule_call(gc, ctx)
    raise GuardError("Unsupported", "unknown clause kind %s" % k)


def eval_when_clause(wc, ctx):
    k = wc["kind"]
    if k == "Clause":
        return eval_guard_access_clause(wc, ctx)
    if k == "NamedRule":
        return eval_guard_named_clause(wc, ctx)
    return eval_parameterized_rule_call(wc, ctx)


def eval_type_block_clause(tb, ctx):
    context = "TypeBlock#%s" % tb["type_name"]
    ctx.start_record(context)
    if tb["conditions"] is not None:
        when_context = "TypeBlock#%s/When" % tb["type_name"]
        ctx.start_record(when_context)
        try:
            st = eval_conjunction_clauses(tb["conditions"], ctx, eval_when_clause)
        except GuardError:
            ctx.end_record(when_context, ("TypeCondition", FAIL))
            ctx.end_record(context, ("TypeCheck", FAIL, tb["type_name"]))
            raise
        if st != PASS:
            ctx.end_record(when_context, ("TypeCondition", st))
            ctx.end_record(context, ("TypeCheck", SKIP, tb["type_name"]))
            return SKIP
        ctx.end_record(when_context, ("TypeCondition", PASS))
    try:
        values = ctx.query(tb["query"])
    except GuardError:
        ctx.end_record(context, ("TypeCheck", FAIL, tb["type_name"]))
        raise
    if not values:
        ctx.end_record(context, ("TypeCheck", SKIP, tb["type_name"]))
        return SKIP
    fails = passes = 0
    for idx, each in enumerate(values):
        if each[0] == "U":
            ctx.end_record(context, ("TypeCheck", FAIL, tb["type_name"]))
            raise GuardError("MissingValue", "Unable to resolve type block query: %s" % tb["type_name"])
        block_context = "%s/%d" % (context, idx)
        ctx.start_record(block_context)
        vr = ValueScope(each[1], ctx)
        try:
            st = eval_general_block_clause(tb["block"], vr, eval_guard_clause)
        except GuardError:
            ctx.end_record(block_context, ("TypeBlock", FAIL))
            ctx.end_record(context, ("TypeCheck", FAIL, tb["type_name"]))
            raise
        if st == PASS:
            passes += 1
        elif st == FAIL:
            fails += 1
        ctx.end_record(block_context, ("TypeBlock", st))
    status = FAIL if fails > 0 else (PASS if passes > 0 else SKIP)
    ctx.end_record(context, ("TypeCheck", status, tb["type_name"]))
    return status


def eval_rule_clause(rc, ctx):
    k = rc["kind"]
    if k == "GuardClause":
        return eval_guard_clause(rc["clause"], ctx)
    if k == "TypeBlock":
        return eval_type_block_clause(rc["type_block"], ctx)
    return eval_when_condition_block("RuleClause", rc["conditions"], rc["block"], ctx)


def eval_rule(rule, ctx):
    context = rule["rule_name"]
    ctx.start_record(context)
    if rule["conditions"] is not None:
        when_context = "Rule#%s/When" % context
        ctx.start_record(when_context)
        try:
            st = eval_conjunction_clauses(rule["conditions"], ctx, eval_when_clause)
        except GuardError:
            ctx.end_record(when_context, ("RuleCondition", FAIL))
            ctx.end_record(context, ("RuleCheck", rule["rule_name"], FAIL, None))
            raise
        if st != PASS:
            ctx.end_record(when_context, ("RuleCondition", st))
            ctx.end_record(context, ("RuleCheck", rule["rule_name"], SKIP, None))
            return SKIP
        ctx.end_record(when_context, ("RuleCondition", PASS))
    try:
        st = eval_general_block_clause(rule["block"], ctx, eval_rule_clause)
    except GuardError:
        ctx.end_record(context, ("RuleCheck", rule["rule_name"], FAIL, None))
        raise
    ctx.end_record(context, ("RuleCheck", rule["rule_name"], st, None))
    return st


def eval_rules_file(rf, ctx, data_file_name):
    context = "File(rules=%d)" % len(rf["guard_rules"])
    ctx.start_record(context)
    fails = passes = 0
    for r in rf["guard_rules"]:
        try:
            st = eval_rule(r, ctx)
        except GuardError:
            ctx.end_record(context, ("RuleCheck", r["rule_name"], FAIL, None))
            raise
        if st == PASS:
            passes += 1
        elif st == FAIL:
            fails += 1
    overall = FAIL if fails > 0 else (PASS if passes > 0 else SKIP)
    ctx.end_record(context, ("FileCheck", data_file_name or "", overall))
    return overall


_DISJ_CONTEXT = {
    "eval_guard_clause": "cfn_guard::rules::exprs::GuardClause#disjunction",
    "eval_when_clause": "cfn_guard::rules::exprs::WhenGuardClause#disjunction",
    "eval_rule_clause": "cfn_guard::rules::exprs::RuleClause#disjunction",
}


def eval_conjunction_clauses(conjunctions, ctx, eval_fn):
    num_passes = num_fails = 0
    # format!("{}#disjunction", std::any::type_name::<T>()) (eval.rs:1980): T from the clause evaluator
    context = _DISJ_CONTEXT[eval_fn.__name__]
    for conjunction in conjunctions:
        disj_fails = 0
        multiple = len(conjunction) > 1
        if multiple:
            ctx.start_record(context)
        passed = False
        for disjunction in conjunction:
            try:
                st = eval_fn(disjunction, ctx)
            except GuardError:
                if multiple:
                    ctx.end_record(context, ("Disjunction", FAIL))
                raise
            if st == PASS:
                num_passes += 1
                if multiple:
                    ctx.end_record(context, ("Disjunction", PASS))
                passed = True
                break
            if st == FAIL:
                disj_fails += 1
        if passed:
            continue
        if disj_fails > 0:
            num_fails += 1
        if multiple:
            ctx.end_record(context, ("Disjunction", FAIL if disj_fails > 0 else SKIP))
    if num_fails > 0:
        return FAIL
    if num_passes > 0:
        return PASS
    return SKIP
