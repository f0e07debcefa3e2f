"""Builds libcfnguard_mi355x.so in-tree (hipcc, --offload-arch=gfx950).

The library holds the host loader/compiler/reporter (C++) and the HIP evaluation kernel; it
links libyaml 0.2.5 (the reference's YAML engine, via unsafe-libyaml) from /opt/conda/lib.

Variants: "" = the product library; "stats" = diagnostic build with evaluator counters
(libcfnguard_mi355x_stats.so, loaded only when GG_LIB points at it); "ab" = an A/B build of the
product sources with extra compile flags from $GG_AB_FLAGS (libcfnguard_mi355x_ab.so).  Every
object records the exact command that produced it (<obj>.cmd), so a flag change rebuilds it.
"""
import os
import shlex
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
HIP_SRCS = ["eval_kernel.hip", "eval_kernel_nfa.hip", "json_gpu.hip", "report_gpu.hip", "order_sort.hip", "capi.cpp"]
# occupancy target of the lane-mode kernel (waves per SIMD); it caps VGPRs at 512 / N.  4 (126 VGPRs,
# 8 spilled) beats 2 (178) and 3 (168): the kernel waits on dependent loads, so resident waves are
# worth more than registers (profiles/r02_ab_occupancy.log; capi.cpp sizes the grid to 16 waves/CU)
LANE_WAVES_PER_EU = os.environ.get("GG_LANE_WAVES_PER_EU", "4")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-I" + YAML_INC, "-Wno-unused-result",
         "-DGG_LANE_WAVES_PER_EU=" + LANE_WAVES_PER_EU]

# Per-source product flags.  MachineLICM hoists loop-invariant immediates (the constant fields of a
# failure record) out of the interpreter loops into callee-saved VGPRs, which every call then saves
# to scratch (99.7 -> 95.8 ms per launch, A/B'd on one box); -O2 instead of -O3 for the evaluator:
# 96.2 -> 94.6 ms (round-1 A/B logs under profiles/r01_ab_*).
# IPRA off: with interprocedural register allocation (this backend's default) the big leaves
# (walk_run, compare_op) clobber callee-saved VGPRs freely and every recursive caller saves all of
# them on entry, whether or not it touches them; without it the allocator keeps the leaves in
# caller-saved registers (cfg-2 60.2 -> 58.5 ms with the query driver inlined, profiles/r02_ab_inline.log).
SRC_FLAGS = {
    "eval_kernel.hip": ["-mllvm", "-disable-machine-licm", "-O2", "-mllvm", "-enable-ipra=false"],
}
SRC_FLAGS["eval_kernel_nfa.hip"] = SRC_FLAGS["eval_kernel.hip"]


def _obj(obj_dir, s):
    return os.path.join(obj_dir, s.replace(".cpp", ".o").replace(".hip", ".o"))


def _includes(path, seen=None):
    """the local headers `path` includes, transitively (#include "x")"""
    import re
    seen = set() if seen is None else seen
    try:
        text = open(path).read()
    except OSError:
        return seen
    for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
        for base in (os.path.dirname(path), CSRC, os.path.join(HERE, "..", "include")):
            cand = os.path.normpath(os.path.join(base, inc))
            if os.path.exists(cand):
                if cand not in seen:
                    seen.add(cand)
                    _includes(cand, seen)
                break
    return seen


def _needs(src, obj, deps, cmd):
    stamp = obj + ".cmd"
    if not os.path.exists(obj) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        if f.read() != " ".join(cmd):
            return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def build(verbose=False, variant=""):
    out = OUT if not variant else OUT.replace(".so", "_" + variant + ".so")
    obj_dir = OBJ if not variant else OBJ + "_" + variant
    flags = list(FLAGS)
    if variant == "stats":
        flags.append("-DGG_STATS")
    elif variant.startswith("ab"):
        pass   # GG_AB_FLAGS go to the evaluator units only (below): an A/B rebuild compiles two files
    elif variant:
        raise ValueError("unknown build variant %r" % variant)
    os.makedirs(obj_dir, exist_ok=True)
    # the units a variant changes (the rest are the product build's objects, shared: the device report
    # alone compiles for ~8 minutes); stats touches every kernel's counters, so it rebuilds everything
    own = None
    if variant.startswith("ab"):
        own = {"eval_kernel.hip", "eval_kernel_nfa.hip"}
    jobs = []
    objs = []
    for s in HOST_SRCS + HIP_SRCS:
        src = os.path.join(CSRC, s)
        if own is not None and s not in own:
            obj = _obj(OBJ, s)
            cmd = [HIPCC, "--offload-arch=gfx950"] + FLAGS + SRC_FLAGS.get(s, []) + ["-c", src, "-o", obj]
        else:
            obj = _obj(obj_dir, s)
            extra = shlex.split(os.environ.get("GG_AB_FLAGS", "")) if variant.startswith("ab") and s.startswith("eval_kernel") else []
            cmd = [HIPCC, "--offload-arch=gfx950"] + flags + SRC_FLAGS.get(s, []) + extra + ["-c", src, "-o", obj]
        objs.append(obj)
        if _needs(src, obj, sorted(_includes(src)), cmd):
            jobs.append((s, obj, cmd))

    def run(job):
        name, obj, cmd = job
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("compile failed: %s\n%s" % (name, r.stderr[-4000:]))
        with open(obj + ".cmd", "w") as f:
            f.write(" ".join(cmd))
        return name

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for name in ex.map(run, jobs):
            if verbose:
                print("compiled", name)
    local_yaml = os.path.join(HERE, "libyaml-0.so.2")
    stale = os.path.exists(out) and any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs if os.path.exists(o))
    if jobs or stale or not os.path.exists(out) or not os.path.exists(local_yaml):
        # libyaml is loaded from the package directory ($ORIGIN): an rpath to /opt/conda/lib would
        # also pull conda's older libstdc++ in front of the one libamdhip64 needs.  Built artefact,
        # not tracked (.gitignore), shipped to the GPU box with the tree.
        shutil.copyfile(os.path.join(YAML_LIB, "libyaml-0.so.2"), local_yaml)
        # linked beside the library and renamed over it: a reader (a test run, a snapshot of the tree) never
        # sees a half-written library
        tmp = out + ".tmp"
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + [
            "-o", tmp, local_yaml, "-Wl,-rpath,$ORIGIN", "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr[-4000:])
        os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(verbose=True, variant=sys.argv[1] if len(sys.argv) > 1 else ""))
    sys.exit(0)
