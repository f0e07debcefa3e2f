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
* Classes like ``\\d``/``\\w``/``\\s`` are Unicode in both engines.
"""
import functools

import regex as _re


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
                    out.append(pattern[i:j + 2])
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
