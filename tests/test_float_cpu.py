"""The device loader's float parser (csrc/eisel_lemire.h: Eisel-Lemire over 128-bit powers of five,
the algorithm of Rust's f64::from_str fast path) run on the host through gg_parse_f64, against
Python's float() -- both correctly rounded, so every accepted number must match bit for bit.  The
parser refuses only infinite results and truncated significands it cannot decide."""
import random
import struct
from fractions import Fraction

import guard_amd


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


EDGE = ["1.5", "-0.0", "0.1", "1e3", "2.5E-3", "123456789012345.0", "1e22", "1e-22", "1e23", "2.2250738585072014e-308",
        "2.2250738585072011e-308", "4.9e-324", "5e-324", "2.4703282292062327e-324", "2.4703282292062328e-324",
        "1.7976931348623157e308", "9007199254740993.0", "0.30000000000000004", "1e-400", "0.1234567890123456789012345",
        "123456789012345678901234567890.5", "9007199254740992.5", "9007199254740993.5", "3.141592653589793238462643"]


def _check(s):
    v = guard_amd.parse_f64(s)
    if v is None:
        # refused only for an infinite result or a significand cut past its 19th digit
        digits = sum(c.isdigit() for c in s.lower().split("e")[0].lstrip("-0."))
        assert float(s) in (float("inf"), float("-inf")) or digits > 19, s
        return 1
    assert _bits(v) == _bits(float(s)), s
    return 0


def test_edge_numbers():
    assert sum(_check(s) for s in EDGE) == 0
    assert guard_amd.parse_f64("1e400") is None            # infinity: the host loader decides
    assert guard_amd.parse_f64("1.7976931348623159e308") is None


def test_random_numbers_match_python():
    rnd = random.Random(11)
    refused = 0
    n = 40000
    for _ in range(n):
        k = rnd.random()
        if k < 0.35:
            s = "%d.%d" % (rnd.randrange(0, 10 ** rnd.randrange(1, 12)), rnd.randrange(0, 10 ** rnd.randrange(1, 12)))
        elif k < 0.65:
            s = "%s%se%d" % (rnd.choice("123456789"), "".join(rnd.choice("0123456789") for _ in range(rnd.randrange(0, 18))),
                             rnd.randrange(-340, 310))
        elif k < 0.9:
            s = "%s.%se%d" % (rnd.choice("123456789"), "".join(rnd.choice("0123456789") for _ in range(rnd.randrange(15, 30))),
                              rnd.randrange(-40, 40))
        else:
            # halfway between two doubles, written out exactly
            m, e = rnd.randrange(2 ** 52, 2 ** 53), rnd.randrange(-30, 30)
            x = Fraction(2 * m + 1) * Fraction(2) ** (e - 1)
            s = format(float(x), ".17g") if rnd.random() < 0.5 else "%d.%s" % (x.numerator // x.denominator, "5")
        if rnd.random() < 0.3:
            s = "-" + s
        refused += _check(s)
    assert refused < n // 20
