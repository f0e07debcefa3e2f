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


def test_native_count_callback_counts_and_accepts():
    # gg_count_write: the measurement sink of the streamed entries (bench --stream-count native)
    fn = ctypes.cast(guard_amd.lib().gg_count_write, guard_amd.WRITE_FN)
    n = ctypes.c_uint64(5)
    buf = ctypes.create_string_buffer(b"abcdef")
    assert fn(ctypes.cast(ctypes.byref(n), ctypes.c_void_p), ctypes.cast(buf, ctypes.c_void_p), 6) == 0
    assert n.value == 11
    assert fn(None, None, 3) == 0


@pytest.mark.skipif(guard_amd.lib().gg_device_available() > 0, reason="GPU present")
def test_no_cpu_fallback():
    with pytest.raises(guard_amd.GuardError) as ei:
        guard_amd.run_checks("{}", "d", "Resources exists", "r")
    assert ei.value.code == -1
    assert "no HIP device" in ei.value.message


def test_c_consumer_builds_and_fails_loudly_without_gpu(tmp_path):
    """A guard-ffi style C program compiles against include/ and links the library unchanged;
    with no GPU in this container it gets code -1 (no CPU fallback)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "cloudformation-guard_amd")
    exe = str(tmp_path / "ffi_run_checks")
    subprocess.check_call(["gcc", os.path.join(root, "examples", "ffi_run_checks.c"), "-I", os.path.join(root, "include"),
                           "-L", pkg, "-lcfnguard_mi355x", "-Wl,-rpath," + pkg, "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    if guard_amd.device_available():   # on a GPU box the same binary evaluates on the device
        assert r.returncode == 0 and '"status": "FAIL"' in r.stdout
    else:
        assert r.returncode == 2
        assert r.stdout.startswith("error: -1 (no HIP device")
