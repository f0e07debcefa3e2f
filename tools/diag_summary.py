"""Prints gpurun_out/diag (kernel_stats.json + bench_files.json) as two tables (diagnostic)."""
import json
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag"
ks = json.load(open(d + "/kernel_stats.json"))
bf = json.load(open(d + "/bench_files.json"))
print("%-46s %7s %6s %6s %6s %6s %6s %5s %5s %5s" % ("file", "ms", "nodes", "heap", "qry", "claus", "frame", "recs", "scan", "ffilt"))
for k, v in ks.items():
    kk = k if k in bf else k[:-len(".guard")]
    print("%-46s %7.3f %6.0f %6.0f %6.0f %6.0f %6.0f %5.1f %5.0f %5.0f" % (
        k[:46], bf[kk]["kernel_ms"], v["node_reads"], v["heap_accesses"], v["query_calls"], v["clause_evals"], v["frames"],
        v["records"], v["map_entries_scanned"], v["fast_filter_tests"]))
T = ["eval_rule", "query_retrieval", "binary_operation", "unary_operation", "rec_push", "filter_test", "resolve_variable",
     "push_frame", "tile_total"]
print("%-46s" % "Kcycles/tile" + "".join("%9s" % t[:8] for t in T))
for k, v in ks.items():
    c = v["cycles_per_tile"]
    print("%-46s" % k[:46] + "".join("%9d" % (c[t] / 1000) for t in T))
