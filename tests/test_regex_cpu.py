"""Rule-regex DFA (csrc/regex_dfa.cpp, run on the host through gg_regex_match) against the oracle's
restatement of Rust regex / fancy-regex `is_match` (oracle/guard_oracle/rxcompat.py), no GPU.

Unicode semantics follow regex-syntax 0.8.5: `\\d` = \\p{Nd}, `\\w` = UTS #18
word characters, `\\s` = \\p{White_Space}, `(?i)` = simple case folding.  Look-around and
back-references must be refused (-1), never approximated.
"""
import json
import os

import pytest

import guard_amd
from guard_oracle import rxcompat

G = os.path.join(os.path.dirname(__file__), "golden")

UNICODE_PATTERNS = [
    r"^\d+$", r"\d", r"^\D+$", r"^\w+$", r"\W", r"^\s+$", r"\S", r"^[\w-]+$", r"^[^\d\s]+$",
    r"(?i)^k$", r"(?i)^s+$", r"(?i)ß", r"(?i)^straße$", r"(?i)σ", r"(?i)^[a-z]+$", r"(?i)[^a-z]",
    r"^.$", r"^..$", r"^\w+@\w+\.\w+$", r"[[:alpha:]]+", r"(?i)[[:upper:]]", r"^[α-ω]+$", r"(?i)^[α-ω]+$",
    r"\x{1F600}", r"^é$", r"^[^a]$", r"a$|^b", r"^$", r"(?i)^ǆ$", r"^\w\s\d$", r"(?s)^a.b$", r"^a.b$",
    r"(foo|bar)+baz", r"^(ab){2,3}$", r"x*", r"\.json$", r"^arn:aws:[a-z0-9-]+:\d{12}:", r"(?i)^(true|false)$",
    # Unicode word boundaries (regex-syntax Look::WordUnicode / WordUnicodeNegate; round 4)
    r"\bfoo\b", r"\b", r"\B", r"^\b", r"\b$", r"\bab", r"ab\b", r"\Bab\B", r"a\B", r"\B\d", r"\b\w+\b",
    r"(?i)\bstraße\b", r"\bé", r"é\b", r"\b(ab|ba)+\b", r"^\B$", r"\b\s", r"(?i)\bTRUE\b|\bfalse\b",
    r"\b[α-ω]+\b", r"x\b|\by", r"\b.\b", r"\B.\B", r"^\bab\b$", r"\b\B", r"(\bfoo)+",
    r"\bprod\b", r"\B\d\B", r"(?i)\bstraße\b|\bσ\w*", r"^\b.\b$|^\B.\B$", r"^\b\w+\b(?:-\b\w+\b)*$", r"\bcafé\b",
]

HAYSTACKS = [
    "", "a", "b", "ab", "ba", "abab", "ababab", "123", "١٢٣", "߀߁", "²", "½", "Ⅻ", "é", "é", "ñandú",
    "straße", "STRASSE", "STRAẞE", "ẞ", "ß", "K", "k", "K", "s", "S", "ſ", "ſſs", "Σ", "σ", "ς",
    "ǅ", "Ǆ", "ǆ", " ", "\t\n", " ", " ", "　", "\x1c", "\x1f", "​", "‍",
    "αβγ", "ΑΒΓ", "😀", "😀😀", "a\nb", "a.b", "a b", "foo@bar.com", "ünïcödé@exämple.org",
    "foobarbaz", "bazfoo", "arn:aws:iam:123456789012:role/x", "template.json", "TRUE", "False", "x_y-z",
    "日本語", "مرحبا", "क्ष", "á", "́",
]


def _patterns():
    return sorted(set(json.load(open(os.path.join(G, "regex_patterns.json"))) + UNICODE_PATTERNS))


@pytest.mark.parametrize("pattern", _patterns())
def test_dfa_matches_oracle(pattern):
    valid = rxcompat.is_valid(pattern)
    rc, states, classes = guard_amd.regex_match(pattern, "x")
    if not valid:
        assert rc in (-1, -2), pattern   # the oracle's engine rejects it; so must the compiler or the path
        return
    if rxcompat.fancy_only(pattern):
        assert rc == -1, pattern         # explicit "unsupported on MI355X path", never approximated
        return
    assert rc in (0, 1), (pattern, rc)
    assert classes < 64 and states < 256, (pattern, states, classes)   # LDS-sized tables
    bad = [(h, guard_amd.regex_match(pattern, h)[0]) for h in HAYSTACKS
           if guard_amd.regex_match(pattern, h)[0] != int(rxcompat.is_match(pattern, h))]
    assert not bad, (pattern, bad)


def test_app_b13_unicode_digits():
    # regex classes are Unicode, `/^\d+$/` matches "١٢٣"
    assert guard_amd.regex_match(r"^\d+$", "١٢٣")[0] == 1
    assert rxcompat.is_match(r"^\d+$", "١٢٣")


# Regexes whose DFA exceeds the compile limits (4000 states / 250 classes) run as the NFA simulation
# (regex_dfa.cpp nfa_fallback, device eval_core.inc nfa_run); the host nfa_match restates the device loop.
_CJK = "".join(chr(0x4E00 + 3 * k) for k in range(260))
NFA_PATTERNS = [
    r"(a|b)*a(a|b){12}", r"^(a|b)*a(a|b){12}$", r"(a|b)*a(a|b){12}$", r"^(a|b)*a(a|b){12}",
    r"(a|b)*a(a|b){12}c", r"x(a|b)*a(a|b){13}|^q", r"(?i)(a|b)*a(a|b){12}",
    "^(" + "|".join(_CJK) + ")+$", "x(" + "|".join(_CJK) + "){2}y", "(" + "|".join(_CJK[:255]) + ")$",
    "[" + _CJK + "]" + "|zz(a|b)*a(a|b){12}",
]


def _nfa_haystacks():
    import random
    r = random.Random(77)
    hs = ["", "a", "b", "c", "q", "x", "y", "zz"]
    for n in (12, 13, 14, 15, 20, 40):
        for _ in range(12):
            hs.append("".join(r.choice("ab") for _ in range(n)))
            hs.append(r.choice(["", "x", "q", "zz"]) + "".join(r.choice("ab") for _ in range(n)) + r.choice(["", "c", "y"]))
    for n in (1, 2, 3, 5):
        for _ in range(10):
            hs.append("".join(r.choice(_CJK + "ab") for _ in range(n)))
            hs.append("x" + "".join(r.choice(_CJK) for _ in range(n)) + "y")
    hs += ["A" * 13, "a" + "B" * 12, "é" + "a" * 13, "日本語", _CJK, _CJK[:2], "\U0001F600" + "a" * 13]
    return hs


@pytest.mark.parametrize("pattern", NFA_PATTERNS)
def test_nfa_fallback_matches_oracle(pattern):
    assert rxcompat.is_valid(pattern) and not rxcompat.fancy_only(pattern)
    assert guard_amd.regex_engine(pattern) == "nfa", pattern
    bad = [(h, rc) for h in _nfa_haystacks()
           for rc in [guard_amd.regex_match(pattern, h)[0]] if rc != int(rxcompat.is_match(pattern, h))]
    assert not bad, (pattern, bad[:5])


def test_nfa_fallback_limits():
    # small regexes keep the DFA; a word assertion in a too-large regex stays refused (-1), never approximated
    assert guard_amd.regex_engine(r"(a|b)*a(a|b){3}") == "dfa"
    assert guard_amd.regex_match(r"\b(a|b)*a(a|b){12}\b", "ab")[0] == -1
    # more than 1024 NFA states: refused
    assert guard_amd.regex_match(r"(a|b)*a(a|b){1100}", "ab")[0] == -1
