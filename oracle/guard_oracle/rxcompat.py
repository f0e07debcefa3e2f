"""Rust ``regex``/``fancy-regex`` matching via the Python ``regex`` module
(TEST INFRASTRUCTURE ONLY -- the parity oracle).

The reference compiles every rule regex with fancy-regex 0.13.0 (over regex 1.11.1 /
regex-syntax 0.8.5, Cargo.lock) and calls ``is_match`` (an unanchored search) at
``guard/src/rules/path_value.rs:255,263,1074-1077``.  Neither crate is vendored in the
reference, so this restates their published semantics on top of the Python ``regex``
module by translating the syntax differences that matter for ``is_match``:

* ``$`` (outside a class, non-multiline) matches only at the very end of the haystack in
  Rust; Python's ``$`` also matches before a trailing newline, so it becomes ``\\Z``.
* ``\\z`` (Rust end of text) becomes ``\\Z``; ``\\A`` is the same in both.
* Perl classes are Unicode in Rust regex-syntax with fixed definitions -- ``\\d`` = ``\\p{Nd}``,
  ``\\w`` = ``[\\p{Alphabetic}\\p{M}\\p{Nd}\\p{Pc}\\p{Join_Control}]`` (UTS #18), ``\\s`` =
  ``\\p{White_Space}`` -- while the Python module's V0 ``\\w`` / ``\\s`` follow ``str.isalnum`` /
  ``str.isspace`` (``\\w`` would take No such as "½" and miss combining marks, ``\\s`` would take
  U+001C..U+001F), so they are spelled out as those property classes.
* ``(?i)`` is simple case folding in both (V0 without FULLCASE).
* ``\\b`` / ``\\B`` are Unicode word boundaries over that same ``\\w`` (regex-syntax
  ``Look::WordUnicode`` / ``WordUnicodeNegate``; the text's ends count as non-word); Python's are over
  its own word definition, so they are spelled out as look-arounds on the spelled-out class.
"""
import functools

import regex as _re


_WORD = r"\p{Alphabetic}\p{M}\p{Nd}\p{Pc}\p{Join_Control}"
# perl class -> (outside a class, inside a class); `\W` inside a class has no V0 spelling (kept)
_W1 = "[" + _WORD + "]"
# \b / \B outside a class: look-arounds on the UTS #18 word class
_BOUNDARY = {"b": "(?:(?<=%s)(?!%s)|(?<!%s)(?=%s))" % (_W1, _W1, _W1, _W1),
             "B": "(?:(?<=%s)(?=%s)|(?<!%s)(?!%s))" % (_W1, _W1, _W1, _W1)}
_PERL = {
    "d": (r"\p{Nd}", r"\p{Nd}"), "D": (r"\P{Nd}", r"\P{Nd}"),
    "s": (r"\p{White_Space}", r"\p{White_Space}"), "S": (r"\P{White_Space}", r"\P{White_Space}"),
    "w": ("[" + _WORD + "]", _WORD), "W": ("[^" + _WORD + "]", None),
}


# regex-syntax ast::ClassAsciiKind (ASCII-only POSIX classes)
_ASCII_CLASSES = {
    "alnum": "0-9A-Za-z", "alpha": "A-Za-z", "ascii": "\\x00-\\x7F", "blank": "\\t ", "cntrl": "\\x00-\\x1F\\x7F",
    "digit": "0-9", "graph": "!-~", "lower": "a-z", "print": " -~", "punct": "!-/:-@\\[-`{-~",
    "space": "\\t\\n\\x0B\\f\\r ", "upper": "A-Z", "word": "0-9A-Za-z_", "xdigit": "0-9A-Fa-f",
}


def translate(pattern: str) -> str:
    out = []
    i = 0
    n = len(pattern)
    in_class = False
    multiline = False
    while i < n:
        c = pattern[i]
        if c == "\\" and i + 1 < n:
            nxt = pattern[i + 1]
            if nxt == "z" and not in_class:
                out.append("\\Z")
            elif nxt in "xuU" and i + 2 < n and pattern[i + 2] == "{":
                # Rust \x{...} / \u{...} / \U{...}: the code point itself
                j = pattern.find("}", i + 3)
                if j < 0:
                    raise ValueError("bad escape")
                out.append(_re.escape(chr(int(pattern[i + 3:j], 16))))
                i = j + 1
                continue
            elif nxt in _BOUNDARY and not in_class:
                out.append(_BOUNDARY[nxt])
            elif nxt in _PERL and not (in_class and nxt == "W"):
                out.append(_PERL[nxt][1 if in_class else 0])
            else:
                out.append(c + nxt)
            i += 2
            continue
        if in_class:
            if c == "]":
                in_class = False
            elif c == "[" and i + 1 < n and pattern[i + 1] == ":":
                j = pattern.find(":]", i + 2)
                if j > 0:
                    # regex-syntax ASCII classes are ASCII-only (Python's are Unicode)
                    name = pattern[i + 2:j]
                    out.append(_ASCII_CLASSES.get(name, pattern[i:j + 2]))
                    i = j + 2
                    continue
            out.append(c)
            i += 1
            continue
        if c == "[":
            in_class = True
            out.append(c)
            i += 1
            # a leading ']' or '^]' is literal
            if i < n and pattern[i] == "^":
                out.append("^")
                i += 1
            if i < n and pattern[i] == "]":
                out.append("\\]")
                i += 1
            continue
        if c == "(" and pattern.startswith("(?", i):
            j = i + 2
            flags = ""
            while j < n and pattern[j] not in ":)":
                flags += pattern[j]
                j += 1
            if "m" in flags.split("-")[0]:
                multiline = True
        if c == "$" and not multiline:
            out.append("\\Z")
            i += 1
            continue
        out.append(c)
        i += 1
    return "".join(out)


@functools.lru_cache(maxsize=4096)
def _compile(pattern: str):
    return _re.compile(translate(pattern), _re.V0)


# Patterns the evaluator actually matched (tests use it to tell which inputs reach a regex).
EVALUATED = set()


def is_match(pattern: str, s: str) -> bool:
    EVALUATED.add(pattern)
    return _compile(pattern).search(s) is not None


def fancy_only(pattern: str) -> bool:
    """constructs only fancy-regex evaluates (look-around, back-references, atomic groups)"""
    import re
    return bool(re.search(r"\(\?<?[=!]|\(\?>|\\[1-9]|\\k<", pattern))


def is_valid(pattern: str) -> bool:
    try:
        _compile(pattern)
        return True
    except Exception:
        return False
