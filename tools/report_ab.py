"""Device JSON report copy-out, session entry against the streamed entry, in one process (diagnostic, GPU):
the same N cfg2 templates rendered by gg_session_report_json_device (counting sink over the session's
staging) and by cfn_guard_validate_batch_stream as one chunk (native counting callback), twice each.
GG_DREPORT_TRACE=1 prints both paths' per-block render / copy spans."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cloudformation-guard_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import guard_amd  # noqa: E402
import rulepack  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
rules = rulepack.rule_pack("cfg2")
texts = guard_amd.SynthTexts(0, n, 50, "json", 16)
for rep in range(2):
    s = guard_amd.Session()
    s.set_option("defer_records", True)
    for name, text in rules:
        s.add_rules(text, name)
    s.add_synthetic_device(0, n, n_resources=50, threads=16)
    s.upload()
    s.eval(1)
    print("[ab] session report start", flush=True, file=sys.stderr)
    t0 = time.time()
    nb, code, st = s.report_json_device()
    dt = time.time() - t0
    s.close()
    print("rep %d session: report %.3f s, %.1f GB/s (d2h_ms %.0f, write_ms %.0f)" % (rep, dt, nb / dt / 1e9, st["d2h_ms"], st["write_ms"]), flush=True)
    print("[ab] stream start", flush=True, file=sys.stderr)
    tot = [0]
    t0 = time.time()
    guard_amd.validate_structured_stream(rules, None, write=lambda k: tot.__setitem__(0, tot[0] + k), chunk_docs=n,
                                         inputs=texts.inputs, n_docs=texts.n, count_only="native")
    dt = time.time() - t0
    print("rep %d stream (load + eval + report): %.3f s, %.1f GB/s of report" % (rep, dt, tot[0] / dt / 1e9), flush=True)
texts.close()
