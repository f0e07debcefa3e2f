"""Host-NUMA placement of the report's pinned staging (diagnostic, GPU): the process's CPUs (and so the
first touch of every host page it allocates, pinned staging included) restricted to NUMA node N before
anything touches the GPU, then the streamed entry on 1M cfg2 texts.  Prints the GPU's node."""
import glob
import os
import sys
import time


def node_cpus(n):
    out = set()
    for part in open("/sys/devices/system/node/node%d/cpulist" % n).read().strip().split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


node = int(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000000
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 262144
gpu_nodes = {}
for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
    try:
        gpu_nodes[p.split("/")[4]] = open(p).read().strip()
    except OSError:
        pass
nodes = sorted(int(os.path.basename(p)[4:]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))
print("numa nodes %s, gpu card nodes %s, pinning to node %d" % (nodes, gpu_nodes, node), flush=True)
if node >= 0:
    os.sched_setaffinity(0, node_cpus(node))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cloudformation-guard_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import guard_amd  # noqa: E402
import rulepack  # noqa: E402
rules = rulepack.rule_pack("cfg2")
t = guard_amd.SynthTexts(0, n, 50, "json", 16)
nb = [0]


def w(k):
    nb[0] += k


t0 = time.time()
_, code = guard_amd.validate_structured_stream(rules, None, write=w, chunk_docs=chunk, inputs=t.inputs, n_docs=t.n,
                                               count_only="native")
dt = time.time() - t0
print("node %d n %d chunk %d: %.3f s, %.1f K evals/s, %.1f GB/s of report" % (node, n, chunk, dt, n * 7 / dt / 1e3,
                                                                              nb[0] / dt / 1e9), flush=True)
t.close()
