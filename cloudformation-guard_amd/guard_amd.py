"""Python host binding (ctypes) for libcfnguard_mi355x.so.

Mirrors the reference's operator interface for the evaluation path:
  * ``run_checks(data, data_name, rules, rules_name)``  <- guard-ffi ``cfn_guard_run_checks``
    (guard-ffi/src/lib.rs:32-45 -> guard/src/commands/helper.rs:25-87)
  * ``validate_structured(rules, data)``                <- ``cfn-guard validate --structured -o json``
    (guard/src/commands/validate.rs:391-403, reporters/validate/structured.rs:99-133)
  * ``Session``                                          batched evaluation with HBM-resident documents

Every call evaluates on the GPU (HIP kernel).  If the shared library has not been built, or no
HIP device is present, calls raise -- there is no CPU fallback.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# GG_LIB selects a diagnostic build variant (e.g. libcfnguard_mi355x_stats.so); default: the product library
LIB_PATH = os.environ.get("GG_LIB") or os.path.join(HERE, "libcfnguard_mi355x.so")


class ExternError(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int32), ("message", ctypes.c_void_p)]


class ValidateInput(ctypes.Structure):
    _fields_ = [("content", ctypes.c_char_p), ("file_name", ctypes.c_char_p)]


class GuardError(Exception):
    def __init__(self, code, message):
        Exception.__init__(self, message)
        self.code = code
        self.message = message


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libcfnguard_mi355x.so is not built (run __graft_entry__.build()); "
                           "the MI355X path has no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    L.cfn_guard_run_checks.argtypes = [ValidateInput, ValidateInput, ctypes.c_bool, ctypes.POINTER(ExternError)]
    L.cfn_guard_run_checks.restype = ctypes.c_void_p
    L.cfn_guard_free_string.argtypes = [ctypes.c_void_p]
    L.cfn_guard_free_string.restype = None
    L.cfn_guard_validate_batch.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.POINTER(ValidateInput),
                                           ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.cfn_guard_validate_batch.restype = ctypes.c_void_p
    L.cfn_guard_validate_batch_format.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                  ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_int32,
                                                  ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.cfn_guard_validate_batch_format.restype = ctypes.c_void_p
    L.cfn_guard_validate_batch_stream.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                  ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_size_t,
                                                  WRITE_FN, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                                  ctypes.POINTER(ExternError)]
    L.cfn_guard_validate_batch_stream.restype = ctypes.c_int32
    if hasattr(L, "cfn_guard_validate_batch_stream_devices"):   # (absent from builds older than round 5: GG_LIB A/B)
        L.cfn_guard_validate_batch_stream_devices.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                              ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                              ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32),
                                                              ctypes.c_size_t, WRITE_FN, ctypes.c_void_p,
                                                              ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
        L.cfn_guard_validate_batch_stream_devices.restype = ctypes.c_int32
    if hasattr(L, "cfn_guard_validate_batch_stream_ex"):   # (round 6: formats and -i on the streamed entries)
        L.cfn_guard_validate_batch_stream_ex.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                         ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                         ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_int32,
                                                         ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t,
                                                         WRITE_FN, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                                         ctypes.POINTER(ExternError)]
        L.cfn_guard_validate_batch_stream_ex.restype = ctypes.c_int32
    L.gg_synth_texts.argtypes = [ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
    L.gg_synth_texts.restype = ctypes.c_void_p
    L.gg_texts_inputs.argtypes = [ctypes.c_void_p]
    L.gg_texts_inputs.restype = ctypes.POINTER(ValidateInput)
    L.gg_texts_free.argtypes = [ctypes.c_void_p]
    L.cfn_guard_validate_batch_params.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                  ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                  ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_int32,
                                                  ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.cfn_guard_validate_batch_params.restype = ctypes.c_void_p
    L.cfn_guard_validate_batch_devices.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                   ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                                   ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_int32,
                                                   ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t,
                                                   ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.cfn_guard_validate_batch_devices.restype = ctypes.c_void_p
    L.gg_shard_by_bytes.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_size_t)]
    L.gg_shard_by_bytes.restype = ctypes.c_int32
    L.gg_session_report_shards.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_size_t),
                                           ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32),
                                           ctypes.POINTER(ExternError)]
    L.gg_session_report_shards.restype = ctypes.c_void_p
    L.gg_session_report_json_device.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32),
                                                ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ExternError)]
    L.gg_session_report_json_device.restype = ctypes.c_int64
    if hasattr(L, "gg_session_report_sarif_device"):
        L.gg_session_report_sarif_device.argtypes = L.gg_session_report_json_device.argtypes
        L.gg_session_report_sarif_device.restype = ctypes.c_int64
    L.gg_session_set_device_report.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.gg_session_set_device_report.restype = ctypes.c_int32
    L.gg_session_set_device.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.gg_session_set_device.restype = ctypes.c_int32
    L.cfn_guard_validate_console.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                             ctypes.POINTER(ValidateInput), ctypes.c_size_t,
                                             ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_uint32,
                                             ctypes.c_int32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32),
                                             ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ExternError)]
    L.cfn_guard_validate_console.restype = ctypes.c_void_p
    L.gg_session_set_params.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                        ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, ctypes.POINTER(ExternError)]
    L.gg_session_set_params.restype = ctypes.c_int32
    L.gg_session_report_range.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.gg_session_report_range.restype = ctypes.c_void_p
    L.gg_session_report_range_n.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t, ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int32),
                                            ctypes.POINTER(ExternError)]
    L.gg_session_report_range_n.restype = ctypes.c_void_p
    L.cfn_guard_test_dir.argtypes = [ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.POINTER(ValidateInput),
                                     ctypes.POINTER(ctypes.c_size_t), ctypes.c_int32, ctypes.c_bool,
                                     ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.cfn_guard_test_ex.argtypes = [ValidateInput, ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_int32,
                                    ctypes.c_bool, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.cfn_guard_test_ex.restype = ctypes.c_void_p
    L.cfn_guard_test_dir.restype = ctypes.c_void_p
    L.gg_session_report_format.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                           ctypes.POINTER(ExternError)]
    L.gg_session_report_format.restype = ctypes.c_void_p
    L.cfn_guard_test.argtypes = [ValidateInput, ctypes.POINTER(ValidateInput), ctypes.c_size_t, ctypes.c_int32,
                                 ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.cfn_guard_test.restype = ctypes.c_void_p
    L.gg_session_new.restype = ctypes.c_void_p
    L.gg_session_free.argtypes = [ctypes.c_void_p]
    L.gg_session_add_rules.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ExternError)]
    L.gg_session_add_docs.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(ExternError)]
    L.gg_session_upload.argtypes = [ctypes.c_void_p, ctypes.POINTER(ExternError)]
    L.gg_session_eval.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ExternError)]
    L.gg_session_report.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ExternError)]
    L.gg_session_report.restype = ctypes.c_void_p
    L.gg_session_stat.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.gg_session_stat.restype = ctypes.c_int64
    L.gg_session_tile_status.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.gg_session_last_kernel_ms.argtypes = [ctypes.c_void_p]
    L.gg_session_last_kernel_ms.restype = ctypes.c_double
    L.gg_device_available.restype = ctypes.c_int32
    L.gg_device_cache_release.argtypes = [ctypes.c_int32]
    L.gg_device_cache_release.restype = ctypes.c_int64
    L.gg_session_set_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.gg_session_set_stream.restype = None
    L.gg_session_launch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ExternError)]
    L.gg_session_wait.argtypes = [ctypes.c_void_p, ctypes.POINTER(ExternError)]
    L.gg_session_wait.restype = ctypes.c_double
    L.gg_session_fetch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ExternError)]
    L.gg_session_ncounts.argtypes = [ctypes.c_void_p]
    L.gg_session_ncounts.restype = ctypes.c_size_t
    L.gg_session_counts_device.argtypes = [ctypes.c_void_p]
    L.gg_session_counts_device.restype = ctypes.c_void_p
    L.gg_session_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.gg_session_configure.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32]
    L.gg_session_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64]
    L.gg_session_set_option.restype = ctypes.c_int32
    L.gg_session_bind_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.gg_session_bind_counts.restype = None
    L.gg_session_drain_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ExternError)]
    L.gg_session_drain_kernel_ms.restype = ctypes.c_size_t
    L.gg_session_kernel_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.gg_synth_cfn_doc.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t]
    L.gg_synth_cfn_doc.restype = ctypes.c_size_t
    L.gg_synth_cfn_yaml_doc.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t]
    L.gg_synth_cfn_yaml_doc.restype = ctypes.c_size_t
    L.gg_session_add_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.POINTER(ExternError)]
    L.gg_session_add_docs_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                             ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ExternError)]
    L.gg_session_add_synthetic_device.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int32,
                                                  ctypes.c_int32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ExternError)]
    L.gg_loader_device_check.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
                                         ctypes.POINTER(ExternError)]
    L.gg_load_dump.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int32, ctypes.POINTER(ExternError)]
    L.gg_load_dump.restype = ctypes.c_void_p
    L.gg_session_add_synthetic_device_fmt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int32,
                                                      ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_double),
                                                      ctypes.POINTER(ExternError)]
    L.gg_parse_rules.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ExternError)]
    L.gg_parse_rules.restype = ctypes.c_int32
    L.gg_regex_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32)]
    L.gg_parse_f64.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_double)]
    L.gg_regex_match.restype = ctypes.c_int32
    L.gg_session_report_bytes.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32),
                                          ctypes.POINTER(ExternError)]
    L.gg_session_report_bytes.restype = ctypes.c_int64
    for fn in (L.gg_session_save_results, L.gg_session_load_results):
        fn.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ExternError)]
        fn.restype = ctypes.c_int32
    L.gg_program_stats.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32)]
    L.gg_program_stats.restype = ctypes.c_int32
    _lib = L
    return L


def program_stats(text, name="r.guard"):
    """Compiled-program sizes (no GPU): blob words, words before the DFA tables, regexes, clauses, parts."""
    out = (ctypes.c_uint32 * 5)()
    rc = lib().gg_program_stats(_b(text), _b(name), out)
    return rc, list(out)


def parse_f64(text):
    """the device loader's float parser on the host: the double, or None when it refuses the number"""
    b = _b(text)
    out = ctypes.c_double(0)
    return out.value if lib().gg_parse_f64(b, len(b), ctypes.byref(out)) == 1 else None


def regex_match(pattern, text):
    """Host run of the rules-file regex DFA (no GPU): (1 / 0 / -1 unsupported / -2 invalid, states, classes)."""
    b = _b(text)
    st = (ctypes.c_uint32 * 2)()
    rc = lib().gg_regex_match(_b(pattern), b, len(b), st)
    return rc, st[0] & 0x7FFFFFFF, st[1]


def regex_engine(pattern):
    """'dfa', or 'nfa' when the regex's DFA exceeds the compile limits and it runs as the NFA simulation."""
    st = (ctypes.c_uint32 * 2)()
    lib().gg_regex_match(_b(pattern), b"", 0, st)
    return "nfa" if st[0] & 0x80000000 else "dfa"


def load_dump(text, mode=0):
    """Host loader diagnostic (no GPU): typed rendering of one document's value tree.
    mode 0 = libyaml loader (CLI path), 1 = serde loader (FFI path)."""
    b = _b(text)
    err = ExternError()
    p = lib().gg_load_dump(b, len(b), mode, ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return _take_string(p)


def parse_rules(text, name="r.guard"):
    """Host rules-file parser diagnostic (no GPU): 0 = rules, 1 = no rules; raises GuardError (code 5)."""
    err = ExternError()
    rc = lib().gg_parse_rules(_b(text), _b(name), ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return rc


LOAD_STATS = ("kernel_ms", "nodes", "distinct_strings", "pool_bytes", "text_bytes", "h2d_ms", "d2h_ms", "table_retries",
              "refused_docs", "gen_ms")


SESSION_OPTIONS = {"rx_memo_per_launch": 1, "defer_records": 2}


def _load_result(rc, err, st):
    if rc < 0:
        _raise(err)
    note = _take_string(err.message)
    if rc == 1:
        return None
    out = dict(zip(LOAD_STATS, list(st)))
    out["note"] = note
    return out


def loader_device_check(texts):
    """1 = the device loader builds the host loader's arena (up to string ids), 0 = differs, -1 = refused;
    returns (verdict, message)"""
    n = len(texts)
    bufs = [_b(t) for t in texts]
    T = (ctypes.c_char_p * n)(*bufs)
    Ls = (ctypes.c_size_t * n)(*[len(b) for b in bufs])
    err = ExternError()
    rc = lib().gg_loader_device_check(T, Ls, n, ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return rc, _take_string(err.message) or ""


def _take_string(p):
    if not p:
        return None
    s = ctypes.string_at(p).decode("utf-8")
    lib().cfn_guard_free_string(p)
    return s


def _owned_bytes(p, n):
    """a uint8 numpy array over n bytes the library malloc'd at p (no copy); freed with the array"""
    import numpy as np
    import weakref
    if not p or n == 0:
        if p:
            lib().cfn_guard_free_string(p)
        return np.zeros(0, dtype=np.uint8)
    buf = (ctypes.c_uint8 * n).from_address(p)
    weakref.finalize(buf, lib().cfn_guard_free_string, p)
    return np.frombuffer(buf, dtype=np.uint8)


def _raise(err):
    msg = _take_string(err.message) or ""
    raise GuardError(err.code, msg)


def _b(s):
    return s.encode("utf-8") if isinstance(s, str) else s


def run_checks(data, data_name, rules, rules_name, verbose=False):
    """guard-ffi run_checks: one document x one rules file -> pretty FileReport JSON (verbose: the
    pretty EventRecord tree of the evaluation, commands/helper.rs:62-64)."""
    err = ExternError()
    p = lib().cfn_guard_run_checks(ValidateInput(_b(data), _b(data_name)), ValidateInput(_b(rules), _b(rules_name)),
                                   verbose, ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return _take_string(p)


# `validate --structured -o <format>` (include/cfn_guard_mi355x.h CFN_GUARD_OUTPUT_*)
OUTPUT_FORMATS = {"json": 0, "yaml": 1, "sarif": 2, "junit": 3}


def validate_structured(rules, data, output="json", params=None):
    """rules: [(name, text)], data: [(name, text)] -> (stdout text, exit_code) for
    `cfn-guard validate --structured -o <output> -S none [-i <params>...]`; params: [(name, text)] in
    the CLI's walk order.  Raises GuardError for an evaluation error (the CLI prints it to stderr, exit -1)."""
    R = (ValidateInput * max(1, len(rules)))(*[ValidateInput(_b(t), _b(n)) for n, t in rules])
    D = (ValidateInput * max(1, len(data)))(*[ValidateInput(_b(t), _b(n)) for n, t in data])
    params = params or []
    P = (ValidateInput * max(1, len(params)))(*[ValidateInput(_b(t), _b(n)) for n, t in params])
    code = ctypes.c_int32(0)
    err = ExternError()
    p = lib().cfn_guard_validate_batch_params(D, len(data), R, len(rules), P, len(params), OUTPUT_FORMATS[output],
                                              ctypes.byref(code), ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return _take_string(p), code.value


WRITE_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


def validate_structured_stream(rules, data, write=None, chunk_docs=0, inputs=None, n_docs=None, count_only=False,
                               devices=False, output="json", params=None):
    """cfn_guard_validate_batch_stream: the JSON report of validate_structured streamed to write(bytes) in
    document order, the documents evaluated in chunks of chunk_docs (0: 262144) on two alternating sessions.
    Returns (text or None, exit_code): the text when write is None (collected), else None.  Raises GuardError on
    an abort (the chunks written before it are a prefix to drop).  inputs / n_docs: a prepared
    ValidateInput array (SynthTexts.inputs) instead of data.  count_only: the text reaches host memory (the
    library's pinned staging) and only its length is taken -- write(n) gets byte counts (measurement); "native":
    the library's counting callback (gg_count_write) takes them, write(total) is called once at the end.
    devices: a list of HIP ordinals (or None: every visible device) for cfn_guard_validate_batch_stream_devices --
    chunk k on devices[k % len(devices)], the same bytes; False (default): the one-device entry.
    output ("json", "yaml", "sarif", "junit") / params ([(name, text)], validate -i): through
    cfn_guard_validate_batch_stream_ex, the one-string call's bytes in every format."""
    R = (ValidateInput * max(1, len(rules)))(*[ValidateInput(_b(t), _b(n)) for n, t in rules])
    if inputs is None:
        inputs = (ValidateInput * max(1, len(data)))(*[ValidateInput(_b(t), _b(n)) for n, t in data])
        n_docs = len(data)
    parts = []
    sink = write if write is not None else parts.append

    def cb(_ctx, ptr, n):
        try:
            sink(n if count_only else ctypes.string_at(ptr, n))
            return 0
        except Exception:
            return 1
    counted = ctypes.c_uint64(0)
    ctx = None
    if count_only == "native":
        # the library's own counting callback (gg_count_write): no Python call per piece; write(total) at the end
        cbf = ctypes.cast(lib().gg_count_write, WRITE_FN)
        ctx = ctypes.cast(ctypes.byref(counted), ctypes.c_void_p)
    else:
        cbf = WRITE_FN(cb)
    code = ctypes.c_int32(0)
    err = ExternError()
    if output != "json" or params:
        P = (ValidateInput * max(1, len(params or [])))(*[ValidateInput(_b(t), _b(n)) for n, t in (params or [])])
        if devices is None:
            devices = list(range(lib().gg_device_available()))
        dv = (ctypes.c_int32 * max(1, len(devices or [])))(*(devices or []))
        lib().cfn_guard_validate_batch_stream_ex(inputs, n_docs, R, len(rules), P, len(params or []), OUTPUT_FORMATS[output],
                                                 chunk_docs, dv if devices else None, len(devices or []), cbf, ctx,
                                                 ctypes.byref(code), ctypes.byref(err))
    elif devices is False:
        lib().cfn_guard_validate_batch_stream(inputs, n_docs, R, len(rules), chunk_docs, cbf, ctx, ctypes.byref(code),
                                              ctypes.byref(err))
    else:
        dv = (ctypes.c_int32 * max(1, len(devices or [])))(*(devices or []))
        lib().cfn_guard_validate_batch_stream_devices(inputs, n_docs, R, len(rules), chunk_docs,
                                                      dv if devices is not None else None, len(devices or []), cbf,
                                                      ctx, ctypes.byref(code), ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    if count_only == "native" and write is not None:
        write(counted.value)
    return (b"".join(parts).decode("utf-8") if write is None else None), code.value


class SynthTexts:
    """synthetic templates generated natively as validate inputs (gg_synth_texts): .inputs, .n"""

    def __init__(self, first, n, n_resources=50, fmt="json", threads=8):
        self.h = lib().gg_synth_texts(first, n, n_resources, {"json": 0, "yaml": 1}[fmt], threads)
        self.inputs = lib().gg_texts_inputs(self.h)
        self.n = n

    def close(self):
        if self.h:
            lib().gg_texts_free(self.h)
            self.h = None


def validate_structured_devices(rules, data, devices=None, output="json", params=None):
    """validate_structured with the documents sharded over HIP devices in this process
    (cfn_guard_validate_batch_devices): contiguous byte-balanced ranges, one per entry of `devices`
    (ordinals may repeat; None: every visible device), reports joined in document order -- the same
    (text, exit_code) as validate_structured."""
    R = (ValidateInput * max(1, len(rules)))(*[ValidateInput(_b(t), _b(n)) for n, t in rules])
    D = (ValidateInput * max(1, len(data)))(*[ValidateInput(_b(t), _b(n)) for n, t in data])
    params = params or []
    P = (ValidateInput * max(1, len(params)))(*[ValidateInput(_b(t), _b(n)) for n, t in params])
    devs = None if devices is None else (ctypes.c_int32 * max(1, len(devices)))(*devices)
    code = ctypes.c_int32(0)
    err = ExternError()
    p = lib().cfn_guard_validate_batch_devices(D, len(data), R, len(rules), P, len(params), OUTPUT_FORMATS[output],
                                               devs, 0 if devices is None else len(devices), ctypes.byref(code),
                                               ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return _take_string(p), code.value


def shard_by_bytes(sizes, nshards):
    """the library's byte-balanced split (gg_shard_by_bytes): [(first, count)] per shard"""
    n = len(sizes)
    L = (ctypes.c_size_t * max(1, n))(*sizes)
    S = (ctypes.c_size_t * (nshards + 1))()
    if lib().gg_shard_by_bytes(L, n, nshards, S) != 0:
        raise ValueError("nshards must be positive")
    return [(S[k], S[k + 1] - S[k]) for k in range(nshards)]


CONSOLE_OUTPUT_FORMATS = {"single-line-summary": 4, "json": 0, "yaml": 1}


def summary_flags(values):
    """--show-summary values folded as Validate::execute does (validate.rs:254-268): `none` resets"""
    st = 0
    for v in values:
        if v == "none":
            st = 0
            continue
        st |= {"pass": 1, "fail": 2, "skip": 4, "all": 7}[v]
    return st


def validate_console(rules, data, summary=("fail",), output="single-line-summary", verbose=False, print_json=False,
                     params=None):
    """`cfn-guard validate` without --structured (console reporters) -> (stdout, exit_code, stderr), the
    oracle's guard_oracle.console.validate_console contract: an evaluation error returns what was written
    before it, exit code -1 and "Error occurred <error>" in stderr; a failure before any evaluation
    (a data or parameter file that does not load) raises GuardError."""
    R = (ValidateInput * max(1, len(rules)))(*[ValidateInput(_b(t), _b(n)) for n, t in rules])
    D = (ValidateInput * max(1, len(data)))(*[ValidateInput(_b(t), _b(n)) for n, t in data])
    params = params or []
    P = (ValidateInput * max(1, len(params)))(*[ValidateInput(_b(t), _b(n)) for n, t in params])
    code = ctypes.c_int32(0)
    etext = ctypes.c_void_p(None)
    err = ExternError()
    flags = (1 if verbose else 0) | (2 if print_json else 0)
    p = lib().cfn_guard_validate_console(D, len(data), R, len(rules), P, len(params), summary_flags(summary),
                                         CONSOLE_OUTPUT_FORMATS[output], flags, ctypes.byref(code), ctypes.byref(etext),
                                         ctypes.byref(err))
    stderr = _take_string(etext.value) if etext.value else ""
    if not p:
        _raise(err)
    if err.code != 0 and err.message:
        lib().cfn_guard_free_string(err.message)
    return _take_string(p), code.value, stderr


TEST_OUTPUT_FORMATS = {"text": 4, "json": 0, "yaml": 1, "junit": 3}


def run_test(rules_text, rules_name, specs, output="text", verbose=False):
    """`cfn-guard test [--verbose]` over one rules file and spec files [(path, text)] -> (report text, exit code)."""
    S = (ValidateInput * max(1, len(specs)))(*[ValidateInput(_b(t), _b(n)) for n, t in specs])
    code = ctypes.c_int32(0)
    err = ExternError()
    p = lib().cfn_guard_test_ex(ValidateInput(_b(rules_text), _b(rules_name)), S, len(specs), TEST_OUTPUT_FORMATS[output],
                                verbose, ctypes.byref(code), ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return _take_string(p), code.value


def run_test_dir(pairs, output="text", verbose=False):
    """`cfn-guard test -d` over [(rules_name, rules_text, [(spec_path, spec_text), ...]), ...] in the
    directory's order -> (report text, exit code)."""
    R = (ValidateInput * max(1, len(pairs)))(*[ValidateInput(_b(t), _b(n)) for n, t, _ in pairs])
    flat = [sp for _, _, sps in pairs for sp in sps]
    S = (ValidateInput * max(1, len(flat)))(*[ValidateInput(_b(t), _b(n)) for n, t in flat])
    C = (ctypes.c_size_t * max(1, len(pairs)))(*[len(sps) for _, _, sps in pairs])
    code = ctypes.c_int32(0)
    err = ExternError()
    p = lib().cfn_guard_test_dir(R, len(pairs), S, C, TEST_OUTPUT_FORMATS[output], verbose, ctypes.byref(code),
                                 ctypes.byref(err))
    if err.code != 0:
        _raise(err)
    return _take_string(p), code.value


class Session:
    """Documents and compiled rules resident in HBM; repeated evaluations for benchmarking."""

    def __init__(self):
        self.s = lib().gg_session_new()

    def close(self):
        if self.s:
            lib().gg_session_free(self.s)
            self.s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_rules(self, text, name):
        err = ExternError()
        lib().gg_session_add_rules(self.s, _b(text), _b(name), ctypes.byref(err))
        if err.code != 0:
            _raise(err)

    def add_docs(self, texts, names=None, mode=0, threads=8):
        n = len(texts)
        bufs = [_b(t) for t in texts]
        T = (ctypes.c_char_p * n)(*bufs)
        Ls = (ctypes.c_size_t * n)(*[len(b) for b in bufs])
        N = (ctypes.c_char_p * n)(*[_b(x) for x in (names or ["" for _ in range(n)])])
        err = ExternError()
        lib().gg_session_add_docs(self.s, T, Ls, N, n, mode, threads, ctypes.byref(err))
        if err.code != 0:
            _raise(err)

    def set_params(self, params):
        """input parameters [(name, text)] merged into every document added afterwards (validate -i)"""
        n = len(params)
        bufs = [_b(t) for _, t in params]
        T = (ctypes.c_char_p * max(1, n))(*bufs)
        Ls = (ctypes.c_size_t * max(1, n))(*[len(b) for b in bufs])
        N = (ctypes.c_char_p * max(1, n))(*[_b(x) for x, _ in params])
        err = ExternError()
        lib().gg_session_set_params(self.s, T, Ls, N, n, ctypes.byref(err))
        if err.code != 0:
            _raise(err)

    def add_docs_device(self, texts, names=None):
        """Parses and interns strict-JSON documents on the MI355X (empty session only).  A document
        outside the device subset is built by the host loader at its position (stats["refused_docs"]
        counts them).  Returns the loader statistics, or None when the batch is refused as a whole
        (a batch-wide limit: nothing loaded)."""
        n = len(texts)
        bufs = [_b(t) for t in texts]
        T = (ctypes.c_char_p * n)(*bufs)
        Ls = (ctypes.c_size_t * n)(*[len(b) for b in bufs])
        N = (ctypes.c_char_p * n)(*[_b(x) for x in (names or ["" for _ in range(n)])])
        st = (ctypes.c_double * len(LOAD_STATS))()
        err = ExternError()
        rc = lib().gg_session_add_docs_device(self.s, T, Ls, N, n, st, ctypes.byref(err))
        return _load_result(rc, err, st)

    def add_synthetic_device(self, first, n, n_resources=50, threads=8, fmt="json"):
        st = (ctypes.c_double * len(LOAD_STATS))()
        err = ExternError()
        rc = lib().gg_session_add_synthetic_device_fmt(self.s, first, n, n_resources, threads, {"json": 0, "yaml": 1}[fmt], st,
                                                        ctypes.byref(err))
        return _load_result(rc, err, st)

    def upload(self):
        err = ExternError()
        lib().gg_session_upload(self.s, ctypes.byref(err))
        if err.code != 0:
            _raise(err)

    def eval(self, iters=1):
        ms = (ctypes.c_double * max(1, iters))()
        err = ExternError()
        lib().gg_session_eval(self.s, iters, ms, ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return list(ms)

    def report(self, output="json"):
        code = ctypes.c_int32(0)
        err = ExternError()
        p = lib().gg_session_report_format(self.s, OUTPUT_FORMATS[output], ctypes.byref(code), ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return _take_string(p), code.value

    def report_range(self, output="json", first=0, count=None):
        """the structured report of documents [first, first + count) alone (a rank's shard)"""
        code = ctypes.c_int32(0)
        err = ExternError()
        n = ctypes.c_size_t(-1).value if count is None else count
        p = lib().gg_session_report_range(self.s, OUTPUT_FORMATS[output], first, n, ctypes.byref(code), ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return _take_string(p), code.value

    def report_range_raw(self, output="json", first=0, count=None):
        """report_range as a uint8 numpy array over the library's buffer: no copy, no decode (bulk
        consumers: the streamed multi-rank gather); the buffer is freed with the array"""
        code = ctypes.c_int32(0)
        ln = ctypes.c_size_t(0)
        err = ExternError()
        n = ctypes.c_size_t(-1).value if count is None else count
        p = lib().gg_session_report_range_n(self.s, OUTPUT_FORMATS[output], first, n, ctypes.byref(ln), ctypes.byref(code),
                                            ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return _owned_bytes(p, ln.value), code.value

    def report_json_device(self, max_docs=0):
        """the JSON report of the first max_docs documents (0: all) rendered on the device, copied to host
        memory and discarded: (bytes, exit code, stats)"""
        code = ctypes.c_int32(0)
        st = (ctypes.c_double * 8)()
        err = ExternError()
        n = lib().gg_session_report_json_device(self.s, max_docs, ctypes.byref(code), st, ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        keys = ("device_docs", "host_docs", "size_ms", "write_ms", "d2h_ms", "host_ms", "body_bytes")
        return n, code.value, dict(zip(keys, list(st)[:7]))

    def report_sarif_device(self, max_docs=0):
        """the SARIF report of the first max_docs documents (0: all): results rendered on the device, copied to
        host memory and discarded: (bytes, exit code, stats)"""
        code = ctypes.c_int32(0)
        st = (ctypes.c_double * 8)()
        err = ExternError()
        n = lib().gg_session_report_sarif_device(self.s, max_docs, ctypes.byref(code), st, ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        keys = ("device_docs", "host_docs", "size_ms", "write_ms", "d2h_ms", "host_ms", "body_bytes", "artifacts")
        return n, code.value, dict(zip(keys, list(st)))

    def set_device_report(self, on):
        """JSON reports rendered on the device (True), on host threads (False), or per GG_DEVICE_REPORT (None)"""
        lib().gg_session_set_device_report(self.s, -1 if on is None else int(bool(on)))

    def report_shards(self, output="json", cuts=()):
        """the report rendered as the shards [0, cuts[0]), [cuts[0], cuts[1]), ... and joined as the
        multi-device entry joins its devices' shards"""
        code = ctypes.c_int32(0)
        err = ExternError()
        C = (ctypes.c_size_t * max(1, len(cuts)))(*cuts)
        p = lib().gg_session_report_shards(self.s, OUTPUT_FORMATS[output], C, len(cuts), ctypes.byref(code),
                                           ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return _take_string(p), code.value

    def set_device(self, device):
        """the session's HIP device (before documents are loaded on / uploaded to a device)"""
        if lib().gg_session_set_device(self.s, device) != 0:
            raise ValueError("set_device after the session holds device state")

    def report_bytes(self, output="json", max_docs=0):
        """renders the report of the first max_docs documents (0: all) in blocks and discards it;
        returns (bytes, exit code)"""
        code = ctypes.c_int32(0)
        err = ExternError()
        n = lib().gg_session_report_bytes(self.s, OUTPUT_FORMATS[output], max_docs, ctypes.byref(code), ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return n, code.value

    def stat(self, what):
        return lib().gg_session_stat(self.s, what)

    def save_results(self, path):
        """diagnostic: the evaluation's tiles / rule statuses / records to a file"""
        err = ExternError()
        lib().gg_session_save_results(self.s, _b(path), ctypes.byref(err))
        if err.code != 0:
            _raise(err)

    def load_results(self, path):
        """diagnostic: results saved by save_results into a session with the same rules and documents
        (renders reports without a GPU)"""
        err = ExternError()
        lib().gg_session_load_results(self.s, _b(path), ctypes.byref(err))
        if err.code != 0:
            _raise(err)

    def tile_status(self, n):
        buf = (ctypes.c_uint8 * n)()
        lib().gg_session_tile_status(self.s, buf, n)
        return bytes(buf)

    def add_synthetic(self, first, n, n_resources=50, threads=8):
        """Appends synthetic templates first..first+n-1 (synth.cfn_doc), generated and loaded natively."""
        err = ExternError()
        lib().gg_session_add_synthetic(self.s, first, n, n_resources, threads, ctypes.byref(err))
        if err.code != 0:
            _raise(err)

    def configure(self, mode=0, lane_heap_bytes=0):
        """mode 0: one tile per lane (+ wave-mode retry of overflowing tiles); 1: one tile per wave."""
        if lib().gg_session_configure(self.s, mode, lane_heap_bytes) != 0:
            raise ValueError("bad session configuration")

    def set_option(self, option, value):
        """gg_session_set_option; option "rx_memo_per_launch": zero the regex memo before every launch"""
        if lib().gg_session_set_option(self.s, SESSION_OPTIONS[option], int(value)) != 0:
            raise ValueError("unknown session option %r" % (option,))

    def set_stream(self, stream_handle):
        lib().gg_session_set_stream(self.s, ctypes.c_void_p(stream_handle))

    def _call(self, fn):
        err = ExternError()
        r = fn(self.s, ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return r

    def launch(self):
        self._call(lib().gg_session_launch)

    def wait(self):
        return self._call(lib().gg_session_wait)

    def fetch(self):
        self._call(lib().gg_session_fetch)

    def ncounts(self):
        return lib().gg_session_ncounts(self.s)

    def counts_device_ptr(self):
        return lib().gg_session_counts_device(self.s)

    def bind_counts(self, dev_ptr, n):
        lib().gg_session_bind_counts(self.s, ctypes.c_void_p(dev_ptr), n)

    def drain_kernel_ms(self, cap=4096):
        buf = (ctypes.c_double * cap)()
        err = ExternError()
        n = lib().gg_session_drain_kernel_ms(self.s, buf, cap, ctypes.byref(err))
        if err.code != 0:
            _raise(err)
        return list(buf)[:min(n, cap)]

    def kernel_stats(self):
        out = (ctypes.c_uint64 * 32)()
        lib().gg_session_kernel_stats(self.s, out, 32)
        return list(out)

    def counts(self):
        n = self.ncounts()
        buf = (ctypes.c_uint64 * max(1, n))()
        lib().gg_session_counts(self.s, buf, n)
        return list(buf)[:n]

    STAT = {"ndocs": 0, "nfiles": 1, "nodes": 2, "bytes": 3, "fail": 4, "pass": 5, "skip": 6, "errors": 7,
            "records": 8, "arena_bytes": 9, "first_error": 10, "record_bytes": 11, "record_cap": 12,
            "max_top": 13, "slots": 14, "heap_bytes": 15, "retried": 16, "lane_slots": 17, "mode": 20,
            "parse_errors": 21, "lane_group": 22, "lane_docs": 23}

    def exit_code(self, output="json"):
        """the structured run's exit code over the evaluated documents, as the report would set it:
        -1 an evaluation error, 19 a FAIL (JUnit keeps 5 when a rules file did not parse), 5 an unparsable
        rules file, else 0 (structured.rs:40-43, 110-112; reporters/mod.rs:97-103)"""
        if self.stat(self.STAT["errors"]) > 0:
            return -1
        parse = self.stat(self.STAT["parse_errors"]) > 0
        if self.stat(self.STAT["fail"]) > 0 and not (output == "junit" and parse):
            return 19
        return 5 if parse else 0


def synth_cfn_yaml_doc(index, n_resources=50):
    """Native synthetic template as block-style YAML (byte-identical to synth.cfn_yaml_doc; no GPU needed)."""
    n = lib().gg_synth_cfn_yaml_doc(index, n_resources, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib().gg_synth_cfn_yaml_doc(index, n_resources, buf, n + 1)
    return buf.value.decode("utf-8")


def synth_cfn_doc(index, n_resources=50):
    """Native synthetic template text (byte-identical to synth.cfn_doc; no GPU needed)."""
    n = lib().gg_synth_cfn_doc(index, n_resources, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib().gg_synth_cfn_doc(index, n_resources, buf, n + 1)
    return buf.value.decode("utf-8")


def device_available():
    return lib().gg_device_available() > 0


def release_device_cache(device=-1):
    """gg_device_cache_release: frees the device blocks the library keeps for reuse (every device with -1);
    returns the bytes released."""
    return int(lib().gg_device_cache_release(device))
