"""Builds libcfnguard_mi355x.so in-tree (hipcc, --offload-arch=gfx950).

The library holds the host loader/compiler/reporter (C++) and the HIP evaluation kernel; it
links libyaml 0.2.5 (the reference's YAML engine, via unsafe-libyaml) from /opt/conda/lib.
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libcfnguard_mi355x.so")
OBJ = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
YAML_INC = "/opt/conda/include"
YAML_LIB = "/opt/conda/lib"

HOST_SRCS = ["doc_loader.cpp", "rules_parser.cpp", "regex_dfa.cpp", "cruet.cpp", "compiler.cpp", "reporter.cpp",
             "synth_corpus.cpp"]
HIP_SRCS = ["eval_kernel.hip", "json_gpu.hip", "capi.cpp"]
# occupancy target of the lane-mode kernel (waves per SIMD); it caps VGPRs at 512 / N
LANE_WAVES_PER_EU = os.environ.get("GG_LANE_WAVES_PER_EU", "2")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-I" + YAML_INC, "-Wno-unused-result",
         "-DGG_LANE_WAVES_PER_EU=" + LANE_WAVES_PER_EU]


# per-source flags of a variant: (variant, source) -> extra flags (a variant not listed for a source
# gets the product flags of that source)
SRC_FLAGS = {
    # MachineLICM hoists loop-invariant immediates (the constant fields of a failure record) out of
    # the interpreter loops into callee-saved VGPRs, which every call then saves to scratch
    # (product default, 99.7 -> 95.8 ms per launch A/B'd on one box); -O2 instead of -O3 for the
    # evaluator: 96.2 -> 94.6 ms (-fno-unroll-loops: 124.9 ms)
    ("", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2"],
    ("stats", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2"],
    # A/B baseline: MachineLICM on
    ("licm", "eval_kernel.hip"): [],
    # codegen experiments on top of the product flags
    ("nounroll", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-fno-unroll-loops"],
    ("o2", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2"],
    # register-allocation experiments around device calls (callee-saved VGPRs go to scratch)
    ("ipra", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2", "-mllvm", "-enable-ipra"],
    ("csr8", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2",
                                  "-mllvm", "-regalloc-csr-first-time-cost=8"],
    ("csr64", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2",
                                   "-mllvm", "-regalloc-csr-first-time-cost=64"],
    # machine-scheduler / wave-priority experiments
    ("silp", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2", "-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    ("smem", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2",
                                  "-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    ("wprio", "eval_kernel.hip"): ["-mllvm", "-disable-machine-licm", "-O2", "-mllvm", "-amdgpu-set-wave-priority"],
}


def _needs(src, obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def build(verbose=False, variant=""):
    """variant "" = the product library; "stats" = diagnostic build with evaluator counters
    (libcfnguard_mi355x_stats.so, loaded only when GG_LIB points at it)."""
    out = OUT if not variant else OUT.replace(".so", "_" + variant + ".so")
    obj_dir = OBJ if not variant else OBJ + "_" + variant
    flags = FLAGS + (["-DGG_STATS"] if variant == "stats" else [])
    if variant.startswith("eu"):   # occupancy experiments: eu<N>[p<W>] = amdgpu_waves_per_eu(N), W-word LDS program window
        eu, _, pw = variant[2:].partition("p")
        flags = [f for f in flags if not f.startswith("-DGG_LANE_WAVES_PER_EU=")] + ["-DGG_LANE_WAVES_PER_EU=" + eu]
        if pw:
            flags.append("-DGG_LDS_PROG_WORDS=" + pw)
    if variant == "iclause":       # call-structure experiments (eval_core.inc CLAUSE_FN / CONJ_FN)
        flags.append("-DGG_INLINE_CLAUSE=1")
    if variant == "iconj":
        flags.append("-DGG_INLINE_CONJ=1")
    if variant.startswith("cpad"):  # Ctx LDS stride experiments: cpad<N> = N pad dwords, cpack<N> = 4 B aligned + N pad dwords
        flags.append("-DGG_CTX_PAD=" + variant[4:])
    if variant.startswith("cpack"):
        flags += ["-DGG_CTX_PACK=1", "-DGG_CTX_PAD=" + variant[5:]]
    if variant.startswith("g"):    # lane-heap interleave experiments: g<N> = 2^N bytes per lane per heap row
        flags.append("-DGG_HEAP_GRAIN=" + variant[1:])
    os.makedirs(obj_dir, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".inc"))]
    headers.append(os.path.join(HERE, "..", "include", "cfn_guard_mi355x.h"))
    jobs = []
    for s in HOST_SRCS + HIP_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(obj_dir, s.replace(".cpp", ".o").replace(".hip", ".o"))
        if _needs(src, obj, headers):
            cmd = [HIPCC, "--offload-arch=gfx950"] + flags + SRC_FLAGS.get((variant, s), SRC_FLAGS.get(("", s), [])) + ["-c", src, "-o", obj]
            jobs.append((s, cmd))

    def run(job):
        name, cmd = job
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("compile failed: %s\n%s" % (name, r.stderr[-4000:]))
        return name

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for name in ex.map(run, jobs):
            if verbose:
                print("compiled", name)
    objs = [os.path.join(obj_dir, s.replace(".cpp", ".o").replace(".hip", ".o")) for s in HOST_SRCS + HIP_SRCS]
    if jobs or not os.path.exists(out):
        # libyaml is loaded from the package directory ($ORIGIN): an rpath to /opt/conda/lib would
        # also pull conda's older libstdc++ in front of the one libamdhip64 needs
        local_yaml = os.path.join(HERE, "libyaml-0.so.2")
        shutil.copyfile(os.path.join(YAML_LIB, "libyaml-0.so.2"), local_yaml)
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + [
            "-o", out, local_yaml, "-Wl,-rpath,$ORIGIN", "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr[-4000:])
    return out


if __name__ == "__main__":
    print(build(verbose=True, variant=sys.argv[1] if len(sys.argv) > 1 else ""))
    sys.exit(0)
