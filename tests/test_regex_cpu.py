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
