"""Device JSON report copy-out rate over repeated reports of one session (diagnostic, GPU): does the
device-to-host rate fall after the first large report, and does an idle pause restore it?"""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cloudformation-guard_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import guard_amd  # noqa: E402
import rulepack  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
pauses = [float(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,0,20,0,60,0").split(",")]
rules = rulepack.rule_pack("cfg2")
s = guard_amd.Session()
s.set_option("defer_records", True)
for name, text in rules:
    s.add_rules(text, name)
s.add_synthetic_device(0, n, n_resources=50, threads=16)
s.upload()
s.eval(1)
for i, p in enumerate(pauses):
    if p:
        time.sleep(p)
    t0 = time.time()
    nb, code, st = s.report_json_device()
    dt = time.time() - t0
    print("report %d after %.0f s idle: %.3f s, %.1f GB/s (d2h_ms %.0f, render kernels %.0f ms)"
          % (i, p, dt, nb / dt / 1e9, st["d2h_ms"], st["write_ms"]), flush=True)
s.close()
