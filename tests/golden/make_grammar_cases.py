"""Builds tests/golden/grammar_cases.json: rule texts from the reference's parser unit tests
(guard/src/rules/parser_tests.rs, v3.1.2) with the accept / reject outcome those tests assert,
lifted to whole rules files so both of our parsers (csrc/rules_parser.cpp through gg_parse_rules,
oracle/guard_oracle/parser.py) can be checked against them.  Run once in the build container:
    python tests/golden/make_grammar_cases.py /root/reference

Also builds tests/golden/parse_error_cases.json: the parse-error messages the reference pins (spans
and contexts its parser tests assert for Failures that reach rules_file unchanged, and the
`cfn-guard test` golden for invalid_rule.guard).

Each case is {"id", "src" (parser_tests.rs line), "how", "text", "accept"}.  `how` says how the
sub-parser input became a rules file:
  file    the text is a whole rules file / rule / type block / assignment already
  clause  a file-level default clause (rules_file -> default_clauses, parser.rs:1867)
  rule    the text wrapped as the body of `rule r { ... }` (rule_block_clause, parser.rs:1704)
  access  `<text> exists` (an access query made into a unary clause)
  let     `let v = <text>` (a value / function call on an assignment's right-hand side)
`accept` is the test's own assertion where it tests at that level ("direct": true), otherwise the
outcome the sub-parser's asserted Ok/Err forces once lifted (a parse that stops before the end of
the input leaves text no top-level item can start with, so the file is rejected).
"""
import json
import os
import re
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = os.path.join(ROOT, "guard", "src", "rules", "parser_tests.rs")


def rust_literal_at(lines, lineno, nth=0):
    """The nth string literal starting on 1-based line `lineno` (raw r#"..."# or escaped "...")."""
    text = "\n".join(lines[lineno - 1:])
    pos = 0
    for _ in range(nth + 1):
        m = re.compile(r'r(#*)"|"').search(text, pos)
        if m.group(0).startswith("r"):
            close = '"' + m.group(1)
            end = text.index(close, m.end())
            val, pos = text[m.end():end], end + len(close)
        else:
            i, out = m.end(), []
            while text[i] != '"':
                if text[i] == "\\":
                    c = text[i + 1]
                    out.append({"n": "\n", "t": "\t", "\\": "\\", '"': '"', "'": "'", "0": "\0"}.get(c, c))
                    i += 2
                else:
                    out.append(text[i])
                    i += 1
            val, pos = "".join(out), i + 1
    return val


def wrap(how, t):
    return {"file": t, "clause": t, "rule": "rule r {\n%s\n}\n" % t, "access": t + " exists",
            "let": "let v = " + t}[how]


def main():
    lines = open(SRC, encoding="utf-8").read().split("\n")
    L = lambda n, k=0: rust_literal_at(lines, n, k)   # noqa: E731
    cases = []

    def add(src, how, text, accept, direct=False):
        cases.append({"id": "L%d_%d" % (src, len(cases)), "src": "parser_tests.rs:%d" % src, "how": how,
                      "text": wrap(how, text), "accept": accept, "direct": direct})

    # -- whole files, rules, type blocks, assignments (asserted Ok by the test itself) ------------
    for n in (3105, 3159, 3276, 3286, 3418, 2728, 3741, 4086, 4430, 3257):
        add(n, "file", L(n), True, True)
    for n in (2474, 2480, 2481):                       # test_type_block
        add(n, "file", L(n), True, True)
    add(4655, "file", L(4655), True, True)             # test_parse_assignment_with_function_call
    add(4673, "file", L(4673), True, True)
    # when-inside-when, asserted as a rule_block_clause; at file level the inner `when` is a
    # GuardClause::WhenBlock (clause, parser.rs:1180-1190), so the file parses too
    add(4017, "rule", L(4017), True, True)
    add(4017, "file", L(4017), True)

    # -- GuardClause::try_from / clause() asserted Ok or Err ------------------------------------
    for n in (3899, 3970, 4010, 3313, 3411, 4150, 4228, 4335, 4368, 3810):
        add(n, "clause", L(n), True, True)
    add(3309, "clause", L(3309), True, True)
    add(3347, "clause", L(3347), True, True)           # this == /\{\{resolve:secretsmanager/
    add(3994, "clause", L(3994), False, True)          # Properties {}
    add(4000, "clause", L(4000), False, True)          # Properties { Statements[*]
    # `not named_rule` is a RuleClause (inside a rule) but not a GuardClause, and default clauses
    # are GuardClauses only (default_clauses, parser.rs:1792-1795)
    add(4409, "rule", L(4409), True, True)
    add(4409, "clause", L(4409), False, True)

    # -- test_clauses / test_rule_clauses bodies inside a rule ----------------------------------
    for k in range(1, 6):
        add(2076, "rule", L(2076, k), True, True)
    for k in (1, 2, 3, 6, 7):
        add(1958, "rule", L(1958, k), True, True)
    add(1958, "rule", "let x = 10\n" + L(1958, 5), True)   # a let, then a plain clause

    # -- test_clause_success (parser_tests.rs:1510-1662): every lhs x op x separator x rhs -----
    seps = [(" ", " "), ("\t", "\n\n\t"), ("\t  ", "\t\t"), (" ", "\n#this comment\n"), (" ", "#this comment\n")]
    bin_ops = [">", "<", "==", "!=", "IN", "!IN", "not IN", "NOT IN"]
    un_ops = ["EXISTS", "!EXISTS", "EMPTY", "NOT EMPTY"]
    for lhs in ("configuration.containers.*.image", "engine"):
        for op in bin_ops:
            for a, b in seps:
                add(1510, "clause", lhs + a + op + b + "PARAMETERS.ImageList", True, True)
        for op in un_ops:
            for a, b in seps:
                add(1556, "clause", lhs + a + op + b, True, True)
                # the unary clause stops before " does.not.error"; the next item cannot start there
                add(1581, "clause", lhs + a + op + b + " does.not.error", False)
    for lhs in ("%engine.port", "%engine.*.image"):
        for op in un_ops:
            for a, b in seps:
                add(1602, "clause", lhs + a + op + b, True, True)
        for rhs in ('"ami-12344545"', "/ami-12/", '["ami-12", "ami-21"]', "{ bare: 10, 'work': 20, 'other': 12.4 }"):
            for op in bin_ops[:6]:
                for a, b in seps:
                    add(1626, "clause", lhs + a + op + b + rhs, True, True)

    # -- test_clause_failures: binary operator without a right-hand side (a cut, parser.rs:1000) -
    for lhs in ("configuration.containers.*.image", "engine"):
        for op in (">", "<", "==", "!="):
            add(1936, "clause", "%s %s << message >>" % (lhs, op), False, True)
    add(1928, "clause", " > 10", False, True)

    # -- test_access / test_var_name_access / test_dotted_access / predicates --------------------
    for t in ("engine", "engine.type", "engine.type.*", "engine.*.type.port", "engine.*.type.%var", "engine[0]",
              "engine [0]", "engine.ok.*", "engine.%name.*", "%engine.type", "%engine.*.type[0]", "%engine.%type.*",
              "%engine.%type.*.port", 'engine[type == "cfn"].port', "%var", "%var_10",
              "x.configuration.engine", "x.*.*.port", "x.port.*.ok", "x.first.0.path",
              "resources", "resources.*.type", "resources.*[ type == /AWS::RDS/ ]"):
        add(945, "access", t, True, True)
    add(1719, "access", L(1719), True, True)
    for t in (".", ".engine", "%_var", "%engine.*.", "x.first. second", "resources.*[]", "resources.*[type == /AWS::RDS/"):
        add(945, "access", t, False)
    add(3856, "access", L(3856), True, True)           # it_support_test
    add(4051, "access", L(4051), True, True)           # is_list_check_parser_bug
    add(4059, "access", L(4059), True, True)           # does_this_work
    add(4504, "access", L(4504), True, True)           # test_variable_capture_syntax
    add(4513, "access", L(4513), True, True)
    add(3151, "access", "%roles.Document", True, True)

    # -- map key filters (test_keys_keyword) -----------------------------------------------------
    for t in ("[KEYS IN %var]", "[KEYS NOT IN %var]", "[KEYS == /aws:S/]", "[KEYS != 'aws:IsSecure']", "[keys !in %var]"):
        add(1320, "access", "Condition" + t, True, True)
    # `[KEYS]` is a map_keys_match Failure (1341) but predicate_or_index tries all_indices first
    # (parser.rs:847-855), which reads it as the capture `[name]` (AllIndices(Some("KEYS")))
    add(1320, "access", "Condition[KEYS]", True)

    # -- operators (test_other_operations, test_value_cmp, unary_parse) ---------------------------
    for t in ("exists", "not exists", "!exists", "!EXISTS", "EMPTY", "NOT EMPTY", 'IN ["t", "n"]', "not in [1]",
              "!in [1]", ">= 5", "<= 5", "> 1", "< 1"):
        add(1212, "clause", "x " + t, True, True)
    for t in ("notexists", "! EMPTY"):
        add(1212, "clause", "x " + t, False, True)
    for t in ("is_string", "IS_STRING", "is_list", "IS_LIST", "is_bool", "IS_BOOL", "is_int", "IS_INT", "IS_FLOAT",
              "is_float", "is_null", "IS_NULL"):
        add(4065, "clause", "x " + t, True, True)

    # -- values on a clause's right-hand side and in lets ----------------------------------------
    for t in ("-124", "12670090", '"Hi there"', "'\"Hi there\"'", "'Hi there'", '"\\"Hi There\\""', "True", "true",
              "False", "false", "12.0", "12e+2", "1.0", "1.5", "/.*PROD.*/", "1234", "12.089", '"String in here"',
              "[]", "[1, 2]", '["hi", "there"]', '[1,       "hi",\n\n3]', "[[1, 2], [3, 4]]",
              "r(10,20)", "r[10, 20)", "r[10, 20]", "r(10.2, 50.5)", "/(\\d{4})-(\\d{2})-(\\d{2})/",
              "/!w\\(?()\"Kuz>/", L(190)):
        add(10, "clause", "x == " + t, True, True)
        add(10, "let", t, True, True)
    for t in ('"\\', "[", "[]]", L(167), "/!w(?()\"Kuz>/", "weifhasidhhfasidf77627&^&*^**", "IiI+L1w="):
        add(30, "clause", "x == " + t, False)
    for n in (324, 332, 338, 342, 345, 361, 397, 414, 534, 538, 542, 560):   # maps, lists of maps, comments
        add(n, "let", L(n), True, True)
    for t in ("count(Resources.*)", L(4545), "substring(%sqs_queues.Arn, 0, 6)"):
        add(4527, "let", t, True, True)

    # -- names (test_var_name, test_type_name) ---------------------------------------------------
    for t in ("v", "var_10", "engine_name", "rule_name_"):
        add(692, "file", "let %s = 1" % t, True, True)
        add(692, "file", "rule %s { x exists }" % t, True, True)
    for t in ("_v", "10"):
        add(692, "file", "let %s = 1" % t, False, True)
        add(692, "file", "rule %s { x exists }" % t, False, True)
    for t in ("AWS::Resource::Type", "Custom::Resource", "AWS::Module::Type::MODULE"):
        add(2430, "file", t + " { x exists }", True, True)
    add(2430, "file", "AWS:: { x exists }", False, True)

    # -- whitespace / comments only: Ok(None) ----------------------------------------------------
    for k in range(3):
        add(589, "file", L(590, k), None, True)
    add(589, "file", L(590, 3), True, True)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "grammar_cases.json")
    json.dump(cases, open(out, "w"), indent=1, ensure_ascii=False)
    print(len(cases), "cases ->", out)
    errors_fixture(lines)


CTX_RHS = 'expecting either a property access "engine.core" or value like "string" or ["this", "that"]'


def display(file, text, off, ctx):
    """Error::ParseError(format!("Parsing Error {ParserError}")) as errors.rs:20,107-115 and
    parser.rs:88-101 display it, for a single-line text (line 1, column = chars before + 1)"""
    return "Parser Error when parsing `Parsing Error Error parsing file %s at line 1 at column %d, when handling %s, " \
           "fragment %s`" % (file, len(text[:off]) + 1, ctx, text[off:])


def errors_fixture(lines):
    """parse-error messages the reference pins: spans + contexts its parser unit tests assert for
    errors that reach the top of rules_file unchanged (Failures: no alt / context() above them),
    and the test command's golden (guard/tests/test_command.rs:183-200)"""
    out = []
    for lhs in ("configuration.containers.*.image", "engine"):   # test_clause_failures 1934-1953
        for op in (">", "<", "==", "!="):
            t = "%s %s << message >>" % (lhs, op)
            out.append({"src": "parser_tests.rs:1936", "file": "g.guard", "text": t,
                        "expected": display("g.guard", t, len(lhs) + len(op) + 1, CTX_RHS)})
    # test_predicate_clause_success #4 / #5 (1865-1878): a Failure out of access()
    t = "resources.*[] exists"
    out.append({"src": "parser_tests.rs:1866", "file": "g.guard", "text": t,
                "expected": display("g.guard", t, len("resources.*["), "There were no clauses present g.guard#1@13")})
    t = "resources.*[type == /AWS::RDS/"
    out.append({"src": "parser_tests.rs:1872", "file": "g.guard", "text": t, "expected": display("g.guard", t, len(t), "")})
    # test_command.rs:183-200: `cfn-guard test` on resources/test-command/rule-dir/invalid_rule.guard
    tc = open(os.path.join(ROOT, "guard", "tests", "test_command.rs"), encoding="utf-8").read()
    i = tc.index("fn test_parse_error_when_guard_rule_has_syntax_error")
    j = tc.index('r#"Parse Error on ruleset file ', i) + len('r#"Parse Error on ruleset file ')
    k = tc.index('"#', j)
    golden = tc[j:k]
    assert golden.endswith("`\n")
    rule = open(os.path.join(ROOT, "guard", "resources", "test-command", "rule-dir", "invalid_rule.guard"),
                encoding="utf-8").read()
    out.append({"src": "test_command.rs:193", "file": "resources/test-command/rule-dir/invalid_rule.guard",
                "text": rule, "expected": golden[:-1]})
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "parse_error_cases.json")
    json.dump(out, open(path, "w"), indent=1, ensure_ascii=False)
    print(len(out), "pinned parse errors ->", path)


if __name__ == "__main__":
    main()
