"""Per-rules-file evaluator counters on the cfg-2 corpus (diagnostic; needs the stats build:
python cloudformation-guard_amd/build.py stats, then GG_LIB=<that .so> python tools/kernel_stats.py N)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import rulepack  # noqa: E402

NAMES = ["node_reads", "heap_accesses", "query_calls", "clause_evals", "frames", "records", "map_entries_scanned",
         "fast_filter_tests"]
ndocs = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
out = {}
for name, text in rulepack.rule_pack():
    s = guard_amd.Session()
    s.add_rules(text, name)
    s.add_synthetic(0, ndocs, threads=16)
    s.upload()
    ms = s.eval(1)
    st = s.kernel_stats()
    tiles = max(1, st[8])
    out[name] = {"kernel_ms": round(min(ms), 3), "tiles": st[8]}
    out[name].update({k: round(st[i] / tiles, 1) for i, k in enumerate(NAMES)})
    s.close()
print(json.dumps(out, indent=1))
