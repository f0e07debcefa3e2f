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
# inclusive shader-clock cycles per tile (outermost entry of each category; lanes of a wave share time)
TIMES = ["eval_rule", "query_retrieval", "binary_operation", "unary_operation", "rec_push", "filter_test",
         "resolve_variable", "push_frame", "tile_total"]
# entries of the noinline evaluator functions per tile (stats slots 18..31; eval_core.inc FCALL)
FCALLS = ["eval_conj", "eval_rule", "block_clause", "type_block", "param_call", "misc_call", "query_retrieval",
          "walk_run", "compare_op", "resolve_variable", "resolve_function", "map_key_filter", "key_var_step",
          "filter_test"]
ndocs = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
out = {}
PACK = os.environ.get("PACK", "cfg2")
if PACK == "micro":
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from micro_cases import CASES  # noqa: E402
    FILES = [(k + ".guard", v) for k, v in CASES.items()]
else:
    FILES = rulepack.rule_pack(PACK)
if os.environ.get("EXTRA"):   # each rule of a variants file on its own (lets first), as tools/rule_split_timing.py
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import re  # noqa: E402
    from rule_split_timing import split_rules  # noqa: E402
    pre, rs = split_rules(open(os.environ["EXTRA"]).read())
    FILES = [(re.match(r"rule (\w+)", r).group(1) + ".guard", "\n".join(pre) + "\n" + r + "\n") for r in rs]
corpus = None
if PACK == "cfg5":
    import synth  # noqa: E402
    corpus = synth.config_corpus(ndocs, start=0)
elif PACK == "cfg4":
    import synth  # noqa: E402
    corpus = synth.tf_corpus(ndocs, n_resources=int(os.environ["SIZE"])) if os.environ.get("SIZE") else synth.tf_bench_corpus(ndocs, start=0)
for name, text in FILES:
    s = guard_amd.Session()
    s.add_rules(text, name)
    if corpus is not None:
        s.add_docs(corpus, ["%s-%d.json" % ("plan" if PACK == "cfg4" else "snapshot", i) for i in range(ndocs)], threads=16)
    else:
        s.add_synthetic(0, ndocs, threads=16)
    s.upload()
    ms = s.eval(1)
    st = s.kernel_stats()
    tiles = max(1, st[8])
    out[name] = {"kernel_ms": round(min(ms), 3), "tiles": st[8]}
    out[name].update({k: round(st[i] / tiles, 1) for i, k in enumerate(NAMES)})
    out[name]["cycles_per_tile"] = {k: round(st[9 + i] / tiles) for i, k in enumerate(TIMES)}
    if len(st) >= 32:
        out[name]["calls_per_tile"] = {k: round(st[18 + i] / tiles, 2) for i, k in enumerate(FCALLS)}
    s.close()
print(json.dumps(out, indent=1))
