"""CPU-side checks of the C ABI: the library loads, exports every symbol include/*.h declares,
and refuses to evaluate without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

import guard_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "cfn_guard_mi355x.h")).read()
    return sorted(set(re.findall(r"\b((?:cfn_guard|gg)_[a-z_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    lib = guard_amd.lib()
    syms = _declared_symbols()
    assert "cfn_guard_run_checks" in syms and "cfn_guard_free_string" in syms
    for s in syms:
        assert hasattr(lib, s), s


def test_free_string_null_is_noop():
    guard_amd.lib().cfn_guard_free_string(None)


@pytest.mark.skipif(guard_amd.lib().gg_device_available() > 0, reason="GPU present")
def test_no_cpu_fallback():
    with pytest.raises(guard_amd.GuardError) as ei:
        guard_amd.run_checks("{}", "d", "Resources exists", "r")
    assert ei.value.code == -1
    assert "no HIP device" in ei.value.message
