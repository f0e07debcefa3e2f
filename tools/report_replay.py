"""Host report-writer profiling without a GPU (diagnostic).
  save (GPU box):  python tools/report_replay.py save OUT.bin NDOCS
  time (any CPU):  python tools/report_replay.py time OUT.bin NDOCS [json|yaml]
The session holds the cfg-2 rule pack and synthetic templates 0..NDOCS-1 (the bench's corpus)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import rulepack  # noqa: E402

mode, path, ndocs = sys.argv[1], sys.argv[2], int(sys.argv[3])
fmt = sys.argv[4] if len(sys.argv) > 4 else "json"
s = guard_amd.Session()
for name, text in rulepack.rule_pack("cfg2"):
    s.add_rules(text, name)
s.add_synthetic(0, ndocs, threads=8)
if mode == "save":
    s.upload()
    s.eval(1)
    s.save_results(path)
    print("saved", path)
else:
    s.load_results(path)
    reps = int(os.environ.get("REPS", "1"))
    for _ in range(reps):
        c0 = os.times()
        t = time.time()
        n, code = s.report_bytes(fmt)
        dt = time.time() - t
        c1 = os.times()
        print("%s: %d bytes in %.3f s = %.3f GB/s (threads %s), exit %d; cpu user %.2f s sys %.2f s" % (
            fmt, n, dt, n / dt / 1e9, os.environ.get("GG_REPORT_THREADS", "auto"), code,
            c1.user - c0.user, c1.system - c0.system))
s.close()
