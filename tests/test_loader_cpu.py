"""Host loader typing pins (no GPU), read from the reference source.

libyaml path (`cfn-guard validate`, guard/src/rules/libyaml/loader.rs:62-119, 227-244), v3.1.2:
plain scalars try i64, then f64 (Rust `str::parse`, so `inf` / `nan` / `1e400` are floats), then
the lowercase-only YAML 1.1 bool words (`is_bool_true` / `is_bool_false`, :103-119), then
`~` / `null` in any case; quoted scalars stay strings; `!!bool` uses `str::parse::<bool>`.
The reference's own test (loader_tests.rs:32-69) only asserts on Bool results, so `Yes` / `TRUE`
staying strings follows from reading :103-119, not from a fixture (SURVEY.md 8(c) skew note).

serde path (guard-ffi `run_checks`, helper.rs:30-42): serde_json, else serde_yaml 0.9 (YAML 1.2
core schema: only true/false in three spellings are bools; u64 past i64 wraps, values.rs:289-293).
"""
import pytest

import guard_amd

LIBYAML = [
    ("yes", "Bool(true)"), ("on", "Bool(true)"), ("y", "Bool(true)"), ("true", "Bool(true)"),
    ("no", "Bool(false)"), ("off", "Bool(false)"), ("n", "Bool(false)"), ("false", "Bool(false)"),
    ("Yes", 'String("Yes")'), ("YES", 'String("YES")'), ("Y", 'String("Y")'), ("True", 'String("True")'),
    ("TRUE", 'String("TRUE")'), ("No", 'String("No")'), ("OFF", 'String("OFF")'), ("N", 'String("N")'),
    ('"yes"', 'String("yes")'), ("'on'", 'String("on")'),
    ("!!bool yes", 'String("yes")'), ("!!bool true", "Bool(true)"), ("!!str 5", 'String("5")'),
    ("~", "Null"), ("null", "Null"), ("NULL", "Null"), ("Null", "Null"),
    ("inf", "Float(inf)"), ("infinity", "Float(inf)"), ("-inf", "Float(-inf)"), ("nan", "Float(NaN)"),
    ("1e400", "Float(inf)"), (".inf", 'String(".inf")'),
    ("0x10", 'String("0x10")'), ("+5", "Int(5)"), ("007", "Int(7)"), ("-0", "Int(0)"), ("1_000", 'String("1_000")'),
    (".5", "Float(0.5)"), ("5.", "Float(5.0)"), ("1e5", "Float(100000.0)"),
    ("9223372036854775807", "Int(9223372036854775807)"), ("9223372036854775808", "Float(9.223372036854776e18)"),
]

SERDE = [
    ("yes", 'String("yes")'), ("on", 'String("on")'), ("y", 'String("y")'), ("no", 'String("no")'),
    ("off", 'String("off")'), ("n", 'String("n")'),
    ("true", "Bool(true)"), ("True", "Bool(true)"), ("TRUE", "Bool(true)"), ("false", "Bool(false)"),
    ("~", "Null"), ("null", "Null"), ("0x10", "Int(16)"), ("+5", "Int(5)"), ("1e5", "Float(100000.0)"),
    ("9223372036854775808", "Int(-9223372036854775808)"),
]


@pytest.mark.parametrize("scalar,want", LIBYAML)
def test_libyaml_plain_scalar_typing(scalar, want):
    assert guard_amd.load_dump("check: " + scalar, 0) == '{"check": %s}' % want


@pytest.mark.parametrize("scalar,want", SERDE)
def test_serde_yaml_scalar_typing(scalar, want):
    assert guard_amd.load_dump("check: " + scalar, 1) == '{"check": %s}' % want


def test_json_words_stay_strings():
    # JSON input quotes these words, so both loaders keep them strings
    for mode in (0, 1):
        assert guard_amd.load_dump('{"a": "yes", "b": "off"}', mode) == '{"a": String("yes"), "b": String("off")}'


def test_duplicate_keys_first_position_last_value():
    # path_value.rs:453-470: MapValue.values is an IndexMap, so a repeated key keeps its first
    # position and takes the last value; MapValue.keys keeps every occurrence with its own mark
    # (the libyaml loader's IndexMap is keyed by (key, Location), loader.rs:172-185)
    assert guard_amd.load_dump("a: 1\nb: 0\na: 2\n", 0) == '{"a": Int(2), "b": Int(0)} keys ["a"@0:0, "b"@1:0, "a"@2:0]'
    assert guard_amd.load_dump("x:\n  - {k: 1, k: 2, j: 3}\n", 0) == '{"x": [{"k": Int(2), "j": Int(3)} keys ["k"@1:5, "k"@1:11, "j"@1:17]]}'
    # no repeated key: no key block
    assert guard_amd.load_dump("a: 1\nb: 0\n", 0) == '{"a": Int(1), "b": Int(0)}'


def test_duplicate_keys_serde_loaders():
    # guard-ffi run_checks: serde_json keeps one key (preserve_order IndexMap, last value, first
    # position); its serde_yaml 0.9 fallback refuses the mapping (DuplicateKeyError) -> code 2
    assert guard_amd.load_dump('{"a": 1, "b": 0, "a": 2}', 1) == '{"a": Int(2), "b": Int(0)}'
    with pytest.raises(guard_amd.GuardError) as ei:
        guard_amd.load_dump("a: 1\nb: 0\na: 2\n", 1)
    assert ei.value.code == 2 and 'duplicate entry with key "a"' in ei.value.message
