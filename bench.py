"""Headline benchmark: (document x rules-file) evaluations/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]; SURVEY.md 8(d) cfg 2): synthetic CloudFormation templates
(50 resources each, synth.cfn_doc; doc i from xorshift32 seed 42 ^ i) x the cfg-2 rule pack
(tests/golden/rulepack: S3/DynamoDB encryption, S3 logging/public-read/SSE, IAM role policies,
EBS encryption; 7 rules files).  Default 1M templates per GPU.

A step = one launch of guard_eval_kernel over every (template, rules file) tile of the rank's
shard, with templates, compiled rules and scratch resident in HBM, followed by the per-rule
PASS/FAIL/SKIP tally kernel (and, for N > 1, the RCCL all-reduce of those tallies -- the only
collective; documents shard with no data-path exchange, so scaling is weak: each rank owns
--docs templates).  Records for failing clauses are written to HBM each step, as the reporter
consumes them.

roofline: HBM-bound.  Algorithmic bytes per launch = arena bytes (nodes x 32 B + string pool +
roots, each template counted once however many rules files read it) + per-tile outputs
(32 B TileOut + 1 B per top-level rule) + record bytes (48 B each).  `achieved` divides that
by the evaluation kernel's mean duration, timed with HIP events on the launch stream (torch's
current stream).  `traffic` is filled from a separate rocprofv3 --pmc pass when
profiles/pmc_<round>.json exists for the same workload, else null.

cpu_baseline: the CPU oracle (oracle/guard_oracle, a pure-Python restatement of the reference
evaluator) run end to end (load + evaluate + structured report) on a bounded sample of the same
templates x the same rule pack, in one process per core on the host cores of this box.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cloudformation-guard_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
DNODE_BYTES = 16          # packed device node (guard_types.h DNodeP)
TILEOUT_BYTES = 32
REC_BYTES = 48


def _cpu_share():
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _oracle_worker(args):
    first, n, n_resources = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import synth
    import rulepack
    from guard_oracle import validate_structured
    rules = rulepack.rule_pack()
    docs = synth.cfn_corpus(n, start=first, n_resources=n_resources)
    t = time.time()
    for i, d in enumerate(docs):
        validate_structured(rules, [("synthetic-%d.json" % (first + i), d)])
    return time.time() - t, n * len(rules)


def cpu_baseline(n_resources, per_core=600):
    import multiprocessing as mp
    cores = _cpu_share()
    ctx = mp.get_context("spawn")
    jobs = [(c * per_core, per_core, n_resources) for c in range(cores)]
    t0 = time.time()
    with ctx.Pool(cores) as pool:
        res = pool.map(_oracle_worker, jobs)
    wall = time.time() - t0
    evals = sum(r[1] for r in res)
    busy = max(r[0] for r in res)
    return {"value": round(evals / busy, 2), "unit": "evals/s", "cores": cores, "kind": "port",
            "sample": "%d synthetic templates x %d rules files (%d evals), oracle end to end (load + evaluate + "
                      "structured report), one process per core; %.1f s wall" % (cores * per_core, evals // max(1, cores * per_core),
                                                                                    evals, wall)}


def load_pmc(workload):
    path = os.path.join(ROOT, "profiles", "pmc_r01.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--docs", type=int, default=1_000_000, help="templates per GPU")
    ap.add_argument("--resources", type=int, default=50)
    ap.add_argument("--threads", type=int, default=0, help="host loader threads (default: CPU share)")
    ap.add_argument("--loader", choices=("host", "device"), default="host",
                    help="document loader: host threads, or the MI355X JSON loader (csrc/json_gpu.hip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-per-core", type=int, default=600)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL); gloo only to rehearse N ranks sharing one GPU (GG_BENCH_DEVICE)")
    args = ap.parse_args()

    import torch
    import guard_amd
    import rulepack
    import sharding

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU baseline runs first, in child processes started before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.resources, args.cpu_per_core)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world)
    # one GPU per rank; GG_BENCH_DEVICE pins every rank to one device (rehearsal on a 1-GPU box)
    torch.cuda.set_device(int(os.environ.get("GG_BENCH_DEVICE", local)))
    if not guard_amd.device_available():
        raise RuntimeError("no HIP device: the MI355X evaluator has no CPU fallback")

    threads = args.threads or _cpu_share()
    rules = rulepack.rule_pack()
    sess = guard_amd.Session()
    for name, text in rules:
        sess.add_rules(text, name)
    t0 = time.time()
    first, count = sharding.shard_range(rank, world, args.docs)
    load_stats = None
    if args.loader == "device":
        load_stats = sess.add_synthetic_device(first, count, n_resources=args.resources, threads=threads)
        if load_stats is None:
            raise RuntimeError("device loader refused the synthetic corpus")
        load_stats["text_GBps"] = round(load_stats["text_bytes"] / (load_stats["kernel_ms"] / 1e3) / 1e9, 2)
    else:
        sess.add_synthetic(first, count, n_resources=args.resources, threads=threads)
    t_load = time.time() - t0
    t0 = time.time()
    sess.upload()
    t_upload = time.time() - t0
    # one non-default stream for the kernels AND the tally all-reduce: torch's default stream has
    # handle 0, which the library reads as "its own stream" -- unordered with the collective
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sess.set_stream(stream.cuda_stream)
    counts = torch.zeros(max(1, sess.ncounts()), dtype=torch.int64, device="cuda")
    sess.bind_counts(counts.data_ptr(), sess.ncounts())

    # warmup: the first full evaluation sizes the record arena (re-runs once if it overflowed)
    sess.eval(1)
    for _ in range(max(0, args.warmup - 1)):
        sess.launch()
    torch.cuda.synchronize()
    sess.drain_kernel_ms()

    ndocs = sess.stat(0)
    nfiles = sess.stat(1)
    ntiles = ndocs * nfiles
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sess.launch()
        sharding.all_reduce_tallies(counts, dist)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms = sess.drain_kernel_ms()
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # statuses + records of the last launch (outside the timed region)
    sess.fetch()
    rec_bytes = sess.stat(11)
    max_top = sess.stat(13)
    arena = sess.stat(9)
    b_alg = arena + ntiles * (TILEOUT_BYTES + max_top) + rec_bytes
    k_mean_ms = sum(kms) / max(1, len(kms))
    achieved = b_alg / (k_mean_ms / 1e3) / 1e9
    tally = sess.counts()
    tally_sum = int(counts.sum().item())   # the all-reduced tensor: every rank's last-step tallies
    n_fail, n_pass, n_skip, n_err = sess.stat(4), sess.stat(5), sess.stat(6), sess.stat(7)

    total_units = ntiles * world * args.steps
    value = total_units / elapsed
    workload = "cfg2: %d synthetic CFN templates/GPU (%d resources) x %d-file rule pack" % (args.docs, args.resources, nfiles)
    if rank == 0:
        traffic = load_pmc(workload)
        line = {
            "metric": "(document x rule) evaluations/sec",
            "value": round(value, 1),
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": workload, "docs_per_gpu": args.docs, "rules_files": nfiles,
                       "tiles_per_gpu": ntiles, "parallelism": "doc-shard x%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic},
            "detail": {"kernel_ms_mean": round(k_mean_ms, 3), "kernel_ms": [round(x, 3) for x in kms],
                       "alg_bytes_per_launch": b_alg, "arena_bytes": arena, "record_bytes": rec_bytes,
                       "nodes": sess.stat(2), "pool_bytes": sess.stat(3),
                       "tiles_fail_pass_skip_err": [n_fail, n_pass, n_skip, n_err],
                       "loader": args.loader, "load_s": round(t_load, 2), "host_threads": threads,
                       "upload_s": round(t_upload, 2), "device_loader": load_stats,
                       "rule_tallies_sum": tally_sum, "rule_tallies_fetched": int(sum(tally))},
        }
        line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    sess.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
