"""Timeline of cfn_guard_validate_batch_stream on the bench's cfg2 texts (diagnostic, GPU)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cloudformation-guard_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import guard_amd
import rulepack
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
mode = sys.argv[3] if len(sys.argv) > 3 else "py"   # py: a Python count callback per piece; native: gg_count_write
rules = rulepack.rule_pack("cfg2")
t = guard_amd.SynthTexts(0, n, 50, "json", 16)
nb = [0]
t0 = time.time()
def w(k):
    nb[0] += k
_, code = guard_amd.validate_structured_stream(rules, None, write=w, chunk_docs=chunk, inputs=t.inputs, n_docs=t.n, count_only=True if mode == "py" else "native")
dt = time.time() - t0
print("n %d chunk %d %s: %.3f s, %.1f K evals/s, %d bytes, exit %d" % (n, chunk, mode, dt, n * 7 / dt / 1e3, nb[0], code), flush=True)
t.close()
