"""Headline benchmark: (document x rules-file) evaluations/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]; SURVEY.md 8(d) cfg 2): synthetic CloudFormation templates
(50 resources each, synth.cfn_doc; doc i from xorshift32 seed 42 ^ i) x the cfg-2 rule pack
(tests/golden/rulepack: S3/DynamoDB encryption, S3 logging/public-read/SSE, IAM role policies,
EBS encryption; 7 rules files).  Default 1M templates per GPU.

A step = one evaluation launch over every (template, rules file) tile of the rank's shard -- the
lane kernel (guard_eval_lanes_kernel: one tile per lane, or for few large documents a group of lanes
per document; tiles that outgrow a lane heap re-run in guard_eval_kernel, one per
wavefront) -- with templates, compiled rules and scratch resident in HBM, followed by the per-rule
PASS/FAIL/SKIP tally kernel (and, for N > 1, the RCCL all-reduce of those tallies -- the only
collective; documents shard with no data-path exchange, so scaling is weak: each rank owns --docs
templates).  Failure records are written to HBM each step, in place, where the device reporter reads
them.

roofline: HBM-bound.  Algorithmic bytes per launch = arena bytes (nodes x 16 B + string pool +
roots, each template counted once however many rules files read it) + per-tile outputs
(32 B TileOut + 1 B per top-level rule) + record bytes (48 B each).  `achieved` divides that
by the evaluation kernel's mean duration, timed with HIP events on the launch stream (torch's
current stream).  `traffic` is filled from a separate rocprofv3 --pmc pass when
profiles/pmc_<round>.json exists for the same workload, else null.

cpu_baseline: the CPU oracle (oracle/guard_oracle, a pure-Python restatement of the reference
evaluator -- NOT the reference binary, which cannot be built here) run on a bounded sample of the
same documents x the same rule pack, in one process per core on the host cores of this box:
`value` end to end (load + evaluate + structured report), `eval_only_value` evaluation alone.  The sample
doubles as a full-size parity check: its per-tile statuses and its structured JSON report (every record,
message and value, digested per core's document range) must equal the ones the GPU session produced for
the same documents inside the full-size launch (`statuses_equal`, `reports_equal`).

e2e (N = 1): the whole job a `validate --structured` user pays for, on the same workload -- load
(synthetic text generated on host threads, then parsed by the MI355X JSON / YAML loader,
csrc/json_gpu.hip, whose arena stays in HBM; --loader host parses on host threads instead), upload
(device packing; PCIe too with the host loader), one evaluation, and the structured JSON report rendered
on the MI355X (csrc/report_gpu.hip) and copied to host memory (report_bytes, discarded) -- the phases
timed one by one and summed (`e2e`); `e2e_stream` times the streamed C-ABI entry a caller uses
(cfn_guard_validate_batch_stream, one wall clock over load, evaluation and report, in a child process),
`e2e_stream_sarif` the same entry writing SARIF (cfn_guard_validate_batch_stream_ex).

--workload: cfg2 (default; BASELINE.json configs[1], the metric's config), cfg3 (the same corpus x
the 22-file full-registry stand-in, configs[2]), cfg4 (Terraform plan JSON with 200-2000
resource_changes and module nesting 6-10 deep x the terraform-infra-related pack, configs[3];
--docs plans, synth.tf_bench_corpus) or cfg5 (AWS Config snapshots x the network-reachability regex /
join pack, configs[4]; --docs snapshots of ~33 CIs each).

Host CPUs: the CPU share of this process -- its affinity set, capped by the pool's per-GPU allotment
when the box declares one (OMP_NUM_THREADS; 16 host CPUs per GPU on the MI355X pool) -- sizes the
cpu_baseline processes, the host loader threads and the report threads; the line names it with the
machine's nproc and CPU model.

Regex memo (DevProg::rx_memo): bench zeroes it before every launch by default
(--rx-memo per-launch), so every timed step pays its own first DFA runs; --rx-memo warm keeps the
library default (zeroed once per upload).
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


def log(msg):
    """progress on stderr (a long phase must keep writing: gpurun takes 3 silent minutes for a hang)"""
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def _cpu_share():
    """host CPUs this process may use: its affinity set, capped by the per-GPU allotment the box declares
    (OMP_NUM_THREADS: 16 per GPU on the MI355X pool, which also bounds worker pools there)"""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def host_info():
    """the host the CPU figures ran on"""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_share": _cpu_share()}


def _workload_docs(workload, first, n, n_resources):
    import synth
    if workload == "cfg5":
        return synth.config_corpus(n, start=first)
    if workload == "cfg4":
        return synth.tf_bench_corpus(n, start=first)
    return synth.cfn_corpus(n, start=first, n_resources=n_resources)


def _oracle_worker(args):
    workload, first, n, n_resources = args
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import rulepack
    from guard_oracle import validate_structured
    from guard_oracle import evaluator as E
    from guard_oracle.loader import load_document
    from guard_oracle.parser import parse_rules
    rules = rulepack.rule_pack(workload)
    docs = _workload_docs(workload, first, n, n_resources)
    # the bench session's document names (bench.py main), so the reports compare byte for byte
    prefix = {"cfg4": "plan", "cfg5": "snapshot"}.get(workload, "synthetic")
    names = ["%s-%d.json" % (prefix, first + i) for i in range(n)]
    outs = []
    t = time.time()
    for name, d in zip(names, docs):
        outs.append(validate_structured(rules, [(name, d)]))
    t_e2e = time.time() - t
    # the structured JSON report of the whole range, joined from the one-document reports (the serde pretty
    # layout: each document's object indented by 2 inside one array), with its exit code
    import hashlib
    joined = "[\n" + ",\n".join(o[0][2:-2] for o in outs) + "\n]"
    codes = [o[1] for o in outs]
    rcode = -1 if -1 in codes else (19 if 19 in codes else 0)
    report = (first, n, hashlib.sha256(joined.encode()).hexdigest(), len(joined), rcode)
    parsed = [load_document(d, name) for name, d in zip(names, docs)]
    prs = [parse_rules(text, rn) for rn, text in rules]
    code = {E.PASS: 0, E.FAIL: 1, E.SKIP: 2}   # guard_types.h ST_PASS / ST_FAIL / ST_SKIP
    st = bytearray()
    t = time.time()
    for name, doc in zip(names, parsed):
        for rf in prs:
            try:
                st.append(code[E.eval_rules_file(rf, E.RootScope(rf, doc), name)])
            except E.GuardError:
                st.append(3)   # an erroring tile (gg_session_tile_status)
    t_eval = time.time() - t
    return t_e2e, t_eval, n * len(rules), first, bytes(st), report


def cpu_baseline(workload, n_resources, per_core):
    import multiprocessing as mp
    cores = _cpu_share()
    ctx = mp.get_context("spawn")
    jobs = [(workload, c * per_core, per_core, n_resources) for c in range(cores)]
    t0 = time.time()
    with ctx.Pool(cores) as pool:
        res = pool.map(_oracle_worker, jobs)
    wall = time.time() - t0
    evals = sum(r[2] for r in res)
    busy = max(r[0] for r in res)
    busy_eval = max(r[1] for r in res)
    # per-(document, rules file) statuses of the sample, tile order: the GPU's are checked against them
    statuses = b"".join(r[4] for r in sorted(res, key=lambda r: r[3]))
    return {"value": round(evals / busy, 2), "unit": "evals/s", "cores": cores, "kind": "port",
            "_statuses": statuses, "_reports": [r[5] for r in sorted(res, key=lambda r: r[3])],
            "eval_only_value": round(evals / busy_eval, 2), "host": host_info(),
            "sample": "%d %s documents x %d rules files (%d evals) through the Python restatement of the reference "
                      "(oracle/guard_oracle, not the reference binary), one process per core; value = load + evaluate + "
                      "structured report, eval_only_value = evaluation alone; %.1f s wall"
                      % (cores * per_core, workload, evals // max(1, cores * per_core), evals, wall)}


def _gen_chunk(args):
    workload, first, n, n_resources = args
    sys.path.insert(0, os.path.join(ROOT, "cloudformation-guard_amd"))
    return _workload_docs(workload, first, n, n_resources)


def generate_docs(workload, first, n, n_resources, procs):
    """document texts of a workload without a native generator (cfg5), in worker processes"""
    import multiprocessing as mp
    step = max(1, (n + procs - 1) // procs)
    jobs = [(workload, first + k, min(step, n - k), n_resources) for k in range(0, n, step)]
    with mp.get_context("spawn").Pool(procs) as pool:
        parts = pool.map(_gen_chunk, jobs)
    return [d for p in parts for d in p]


def _stream_leg(workload, first, docs, resources, fmt, chunk, devices, threads, output="json"):
    """a streamed C-ABI leg in a child process (tools/stream_leg.py): the entry as a caller process uses it, with
    none of this process's sessions, caches or copy queues; the child is started, not exec'd"""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "tools", "stream_leg.py"), workload, str(first), str(docs), str(resources),
           fmt, str(chunk), str(devices), str(threads), output]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError("stream leg failed (%d): %s" % (r.returncode, r.stderr[-2000:]))
    return json.loads(r.stdout.strip().splitlines()[-1])


def load_pmc(workload):
    """HBM bytes per launch of the dominant kernel from the newest profiles/pmc_r<NN>.json recorded for
    this exact workload (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes), else None"""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_r*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("cfg2", "cfg3", "cfg4", "cfg5"), default="cfg2")
    ap.add_argument("--docs", type=int, default=0, help="documents per GPU (default: 1M templates; cfg4 8192 plans; "
                                                         "cfg5 303031 snapshots = 10M configuration items)")
    ap.add_argument("--mode", choices=("auto", "lane", "wave"), default="auto",
                    help="evaluation kernel: one tile per lane (+ wave-mode retry), one tile per wavefront, or the "
                         "library's choice (gg_session_configure)")
    ap.add_argument("--reporter", choices=("device", "host"), default="device",
                    help="e2e: the structured JSON report rendered on the MI355X (csrc/report_gpu.hip) and copied to "
                         "host memory, or rendered by the host writer on host threads")
    ap.add_argument("--rx-memo", choices=("per-launch", "warm"), default="per-launch",
                    help="regex is_match memo: zeroed before every launch, or kept warm across launches")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--e2e-sarif", type=int, default=1, help="also time the e2e job with the SARIF report (device results)")
    ap.add_argument("--e2e-stream", type=int, default=262144,
                    help="also time the streamed batch entry (cfn_guard_validate_batch_stream) over the same synthetic "
                         "texts with this many documents per chunk (0: off; cfg2/cfg3 at N=1 only)")
    ap.add_argument("--e2e-stream-runs", type=int, default=2,
                    help="runs of the streamed JSON leg (a child process each); the line reports the fastest and lists all")
    ap.add_argument("--e2e-devices-docs", type=int, default=262144,
                    help="also time the streamed batch entry over every visible device (cfn_guard_validate_batch_stream_"
                         "devices) with this many synthetic documents per device (0: off; cfg2/cfg3 at N=1 only)")
    ap.add_argument("--e2e-devices-chunk", type=int, default=16384, help="documents per chunk of the multi-device stream")
    ap.add_argument("--e2e-report-docs", type=int, default=0,
                    help="documents whose structured report is rendered for e2e (0: all, the default); a sample's "
                         "report time is scaled to the whole job")
    ap.add_argument("--resources", type=int, default=50)
    ap.add_argument("--format", choices=("json", "yaml"), default="json",
                    help="cfg2/cfg3 synthetic templates as JSON, or as block-style CloudFormation YAML "
                         "(synth.cfn_yaml_doc; the device YAML loader, csrc/yaml_gpu.inc)")
    ap.add_argument("--threads", type=int, default=0, help="host loader threads (default: CPU share)")
    ap.add_argument("--loader", choices=("device", "host"), default="device",
                    help="document loader: the MI355X JSON loader (csrc/json_gpu.hip; documents outside its "
                         "subset are built on host threads), or host threads only")
    ap.add_argument("--gather-docs", type=int, default=-1,
                    help="N > 1: the structured JSON report of each rank's first GATHER_DOCS documents (-1: all, the "
                         "default; 0: none) streamed to rank 0 in blocks (sharding.stream_report; outside the timed "
                         "region), where a counting sink consumes it")
    ap.add_argument("--gather-block", type=int, default=4096, help="documents per streamed report block")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-per-core", type=int, default=0)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL); gloo only to rehearse N ranks sharing one GPU (GG_BENCH_DEVICE)")
    args = ap.parse_args()
    if not args.docs:
        args.docs = {"cfg5": 303_031, "cfg4": 8192}.get(args.workload, 1_000_000)
    if not args.cpu_per_core:
        args.cpu_per_core = {"cfg2": 400, "cfg3": 120, "cfg4": 2, "cfg5": 600}[args.workload]

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
        log("cpu baseline (%s, %d documents per core)" % (args.workload, args.cpu_per_core))
        cpu = cpu_baseline(args.workload, args.resources, args.cpu_per_core)
        log("cpu baseline: %s evals/s" % cpu["value"])
    first, count = sharding.shard_range(rank, world, args.docs)
    # The streamed C-ABI legs (N = 1) run next, each in a child process of its own, before this process touches
    # the GPU: a caller of the entry holds no other session, cached blocks or copy queues.  Run after this
    # process's own 1 M-document session and its 149 GB e2e report (as in round 5), the same JSON leg took 7.7 s
    # against 5.3 s standalone on one box (profiles/r06zc_bench_cfg2.json, r06zd_stream_trace.log).
    early = {}
    if (rank == 0 and world == 1 and not args.no_e2e and args.workload in ("cfg2", "cfg3") and args.loader == "device"):
        lthreads = args.threads or _cpu_share()
        legs = []
        if args.e2e_stream:
            legs.append(("json", count, args.e2e_stream, 0, "json"))
            if args.e2e_sarif:
                legs.append(("sarif", count, args.e2e_stream, 0, "sarif"))
        if args.e2e_devices_docs:
            legs.append(("devices", args.e2e_devices_docs, args.e2e_stream, 1, "json"))
        for key, nd, chunk, ndev, output in legs:
            # the JSON leg runs --e2e-stream-runs times (a process each) and reports the fastest with every run's
            # wall clock: the same leg took 5.0-12.8 s on one box from run to run (profiles/r06zk_*, r06zm_*)
            runs = max(1, args.e2e_stream_runs) if key == "json" else 1
            for r in range(runs):
                log("e2e stream leg %s (run %d/%d): %d documents in chunks of %d (a process of its own)"
                    % (key, r + 1, runs, nd, chunk))
                try:
                    leg = _stream_leg(args.workload, first, nd, args.resources, args.format, chunk, ndev, lthreads, output)
                except Exception as e:   # the leg is reported as failed; the line still prints
                    early[key] = {"error": str(e)[-500:]}
                    break
                all_s = early.get(key, {}).get("runs_s", []) + [round(leg["seconds"], 3)]
                if key not in early or leg["seconds"] < early[key]["seconds"]:
                    early[key] = leg
                early[key]["runs_s"] = all_s
    texts = None
    t_gen = 0.0
    if args.workload in ("cfg4", "cfg5"):
        log("generate %d %s documents" % (count, args.workload))
        t0 = time.time()
        texts = generate_docs(args.workload, first, count, args.resources, _cpu_share())
        t_gen = time.time() - t0
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
    rules = rulepack.rule_pack(args.workload)
    sess = guard_amd.Session()
    if args.mode != "auto":
        sess.configure(mode=1 if args.mode == "wave" else 0)
    sess.set_option("rx_memo_per_launch", args.rx_memo == "per-launch")
    # the records stay in HBM where the evaluation wrote them: the device reporter reads them in place, so
    # nothing is compacted after a launch (host writers would compact and copy them on demand)
    sess.set_option("defer_records", args.reporter == "device")
    for name, text in rules:
        sess.add_rules(text, name)
    log("load %d documents" % count)
    t0 = time.time()
    load_stats = None
    n_ci = 0
    if texts is not None:
        prefix = "snapshot" if args.workload == "cfg5" else "plan"
        names = ["%s-%d.json" % (prefix, first + i) for i in range(count)]
        if args.workload == "cfg5":
            n_ci = sum(t.count('"configurationItemStatus"') for t in texts)
        n_changes = sum(t.count('"change":{') for t in texts) if args.workload == "cfg4" else 0
        load_stats = sess.add_docs_device(texts, names) if args.loader == "device" else None
        if load_stats is None:
            # host loader threads: --loader host, or a batch the device parse refuses as a whole (too few,
            # large documents for one lane per document: cfg4's plans)
            if args.loader == "device":
                log("device loader refused the %s batch: host loader threads" % args.workload)
            sess.add_docs(texts, names, threads=threads)
        texts = None
    elif args.loader == "device":
        load_stats = sess.add_synthetic_device(first, count, n_resources=args.resources, threads=threads, fmt=args.format)
        if load_stats is None:
            raise RuntimeError("device loader refused the synthetic corpus")
        t_gen = load_stats["gen_ms"] / 1e3
    else:
        sess.add_synthetic(first, count, n_resources=args.resources, threads=threads)
    if load_stats is not None:
        load_stats["text_GBps"] = round(load_stats["text_bytes"] / (load_stats["kernel_ms"] / 1e3) / 1e9, 2)
    t_load = time.time() - t0
    log("upload (load %.1f s)" % t_load)
    t0 = time.time()
    sess.upload()
    t_upload = time.time() - t0
    log("warmup")
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
    t0 = time.time()
    sess.fetch()
    t_fetch = time.time() - t0
    rec_bytes = sess.stat(11)
    max_top = sess.stat(13)
    arena = sess.stat(9)
    b_alg = arena + ntiles * (TILEOUT_BYTES + max_top) + rec_bytes
    k_mean_ms = sum(kms) / max(1, len(kms))
    achieved = b_alg / (k_mean_ms / 1e3) / 1e9
    tally = sess.counts()
    if cpu is not None and first == 0:
        # the CPU baseline's sample is the first documents of this corpus: their (document, rules file)
        # statuses from the oracle must equal the GPU's, tile for tile
        exp = cpu.pop("_statuses")
        got = sess.tile_status(len(exp))
        bad = [i for i in range(len(exp)) if exp[i] != got[i]]
        cpu["statuses_checked"] = len(exp)
        cpu["statuses_equal"] = not bad
        if bad:
            cpu["first_mismatch_tile"] = bad[0]
            log("CPU/GPU status MISMATCH at %d of %d tiles (first: tile %d)" % (len(bad), len(exp), bad[0]))
        # and their structured JSON reports (records, messages, values: every byte), rendered from the
        # full-size session's results for the same document ranges
        reps = cpu.pop("_reports", [])
        if args.format == "json" and reps and args.workload in ("cfg2", "cfg3", "cfg4", "cfg5"):
            import hashlib
            t0 = time.time()
            mism = []
            for (f0, n, digest, nbytes, code) in reps:
                txt, gcode = sess.report_range("json", f0, n)
                if gcode != code or len(txt) != nbytes or hashlib.sha256(txt.encode()).hexdigest() != digest:
                    mism.append(f0)
            cpu["reports_checked_docs"] = sum(r[1] for r in reps)
            cpu["reports_equal"] = not mism
            cpu["reports_check_s"] = round(time.time() - t0, 2)
            if mism:
                cpu["first_report_mismatch_range"] = mism[0]
                log("CPU/GPU report MISMATCH in %d of %d document ranges (first at document %d)" % (len(mism), len(reps), mism[0]))
    elif cpu is not None:
        cpu.pop("_statuses", None)
        cpu.pop("_reports", None)
    tally_sum = int(counts.sum().item())   # the all-reduced tensor: every rank's last-step tallies
    n_fail, n_pass, n_skip, n_err = sess.stat(4), sess.stat(5), sess.stat(6), sess.stat(7)

    gather = None
    if world > 1 and args.gather_docs != 0:
        # the report half of the multi-GPU path: every rank renders its documents' reports
        # in blocks, rank 0 receives them over the collective backend (RCCL: device buffers) in rank order
        # and joins them into the job's report as they arrive -- here into a sink that counts the bytes
        gdocs = ndocs if args.gather_docs < 0 else min(ndocs, args.gather_docs)

        class _CountingSink:
            n = 0
            last = 0.0

            def write(self, piece):
                self.n += len(piece)
                if time.time() - self.last > 20:
                    self.last = time.time()
                    log("gather: %.1f GB at rank 0" % (self.n / 1e9))

        sink = _CountingSink() if rank == 0 else None
        log("gather: streaming the JSON report of %d documents per rank to rank 0" % gdocs)
        dist.barrier()
        t0 = time.time()
        job_code, gerr = sharding.stream_report(lambda f, c: sess.report_range_raw("json", f, c)[0], gdocs,
                                                sess.exit_code("json"), dist, sink, output="json",
                                                block_docs=args.gather_block, raw=True)
        t_gather = time.time() - t0
        if rank == 0:
            gather = {"docs_per_rank": gdocs, "docs": gdocs * world, "block_docs": args.gather_block,
                      "gather_s": round(t_gather, 3), "bytes": sink.n,
                      "GBps_at_rank0": round(sink.n / max(t_gather, 1e-9) / 1e9, 3), "exit_code": job_code,
                      "error": gerr}

    e2e = None
    e2e_sarif = None
    if rank == 0 and world == 1 and not args.no_e2e:
        rdocs = min(ndocs, args.e2e_report_docs) if args.e2e_report_docs else ndocs
        log("e2e: structured report of %d of %d documents" % (rdocs, ndocs))
        t0 = time.time()
        os.environ.setdefault("GG_PROGRESS", "1")   # a block line per 65536 documents (a long render keeps writing)
        rep_stats = None
        if args.reporter == "device":
            rep_bytes, rep_code, rep_stats = sess.report_json_device(rdocs)
        else:
            rep_bytes, rep_code = sess.report_bytes("json", rdocs)
        t_report_sample = time.time() - t0
        # the synthetic documents are alike: the whole report costs ndocs / rdocs times the sample
        t_report = t_report_sample * ndocs / max(1, rdocs)
        t_eval = k_mean_ms / 1e3 + t_fetch
        # the documents' text is the job's input, resident in host memory when the job starts (a user's
        # files): synthetic text generation is reported apart (gen_s), not counted in load_s -- except
        # with --loader host on cfg2/3, where the native generator runs inside the host loader's threads
        gen_in_load = args.loader == "host" and args.workload in ("cfg2", "cfg3")
        t_load_job = t_load - (t_gen if (args.loader == "device" and args.workload in ("cfg2", "cfg3")) else 0.0)
        total = t_load_job + t_upload + t_eval + t_report
        e2e = {"value": round(ntiles / total, 1), "unit": "evals/s", "load_s": round(t_load_job, 3),
               "gen_s": round(t_gen, 3), "gen_in_load": gen_in_load,
               "upload_s": round(t_upload, 3), "eval_fetch_s": round(t_eval, 3), "report_s": round(t_report, 3),
               "report_docs_rendered": rdocs, "report_s_rendered": round(t_report_sample, 3),
               "report_bytes_rendered": rep_bytes, "report_GBps": round(rep_bytes / t_report_sample / 1e9, 3),
               "exit_code": rep_code, "report_threads": threads, "reporter": args.reporter,
               "device_reporter": rep_stats,
               "pcie_inclusive_value": round(ntiles / (t_upload + t_eval), 1),
               "note": "one job over input text resident in host memory: load (%s) + upload + one evaluation with "
                       "statuses/records fetched + structured JSON report rendered (reporter: device or host) and discarded "
                       "(rendered for report_docs_rendered documents; report_s scaled to all when that is fewer; "
                       "reporter=device: rendered on the MI355X and copied to host memory in blocks); "
                       "synthetic text generation (gen_s) is not part of the job%s"
                       % (("device %s loader: text H2D, parse, intern index to the host (the arena stays in HBM)" % args.format.upper()) if args.loader == "device"
                          else "host loader threads", " (inside load_s with --loader host)" if gen_in_load else "")}

        if args.reporter == "device" and args.e2e_sarif and hasattr(sess, "report_sarif_device"):
            # the same job with the SARIF report (row N2): artifacts and frame on the host, every FAILed
            # document's results rendered on the device from the same records, copied out and counted
            t0 = time.time()
            sr_bytes, sr_code, sr_stats = sess.report_sarif_device(rdocs)
            t_sr_sample = time.time() - t0
            t_sr = t_sr_sample * ndocs / max(1, rdocs)
            e2e_sarif = {"value": round(ntiles / (t_load_job + t_upload + t_eval + t_sr), 1), "unit": "evals/s",
                         "report_s": round(t_sr, 3), "report_bytes_rendered": sr_bytes,
                         "report_GBps": round(sr_bytes / t_sr_sample / 1e9, 3), "exit_code": sr_code,
                         "device_reporter": sr_stats,
                         "note": "e2e with -o sarif: load, upload and evaluation as e2e, the SARIF report rendered on "
                                 "the device (results) and host (artifacts, frame), copied to host memory and discarded"}

    # the session's counters for the line, then its device memory back (the streamed legs run in a child
    # process next to this one: they get the device this process no longer needs)
    sess_stats = {"nodes": sess.stat(2), "pool_bytes": sess.stat(3), "retried": sess.stat(16), "mode": sess.stat(20)}
    sess.close()
    sess = None
    if rank == 0:
        guard_amd.release_device_cache(-1)
        counts = None
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    e2e_stream = None
    leg = None
    if (rank == 0 and world == 1 and not args.no_e2e and args.e2e_stream and args.workload in ("cfg2", "cfg3")
            and args.loader == "device"):
        # the drop-in batch entry end to end: cfn_guard_validate_batch_stream over the same templates as
        # validate inputs, chunks of --e2e-stream documents on two alternating sessions (the next chunk's text
        # H2D, parse and evaluation overlap this chunk's device render and report D2H); the bytes reach host
        # memory (the library's pinned staging) and are counted
        leg = early.get("json")
    if e2e_stream is None and leg is not None and "error" in leg:
        e2e_stream = {"value": None, "error": leg["error"]}
    elif leg is not None:
        t_stream, t_gen_s, st_code = leg["seconds"], leg["gen_s"], leg["exit_code"]
        nbytes = [leg["report_bytes"]]
        e2e_stream = {"value": round(ntiles / t_stream, 1), "unit": "evals/s", "seconds": round(t_stream, 3),
                      "chunk_docs": args.e2e_stream, "report_bytes": nbytes[0],
                      "report_GBps": round(nbytes[0] / t_stream / 1e9, 3), "exit_code": st_code,
                      "gen_s": round(t_gen_s, 3), "runs_s": leg.get("runs_s"),
                      "note": "cfn_guard_validate_batch_stream (the C ABI batch entry, JSON) in a process of its own over "
                              "the same synthetic texts resident in host memory: load + upload + evaluation + fetch + "
                              "device-rendered report to host memory (shader copy-out), chunked and overlapped, counted "
                              "by the library's native callback; text generation (gen_s) not included; the fastest of "
                              "runs_s (one process each, before the bench process touches the GPU)"}

    e2e_stream_sarif = None
    if (rank == 0 and world == 1 and not args.no_e2e and args.e2e_stream and args.e2e_sarif
            and args.workload in ("cfg2", "cfg3") and args.loader == "device"):
        # the same streamed entry writing SARIF (cfn_guard_validate_batch_stream_ex): every chunk evaluated and held
        # on the device, the artifacts written, then each chunk's device-rendered results in order
        try:
            sl = early.get("sarif") or {"error": "not run"}
            if "error" in sl:
                raise RuntimeError(sl["error"])
            e2e_stream_sarif = {"value": round(ntiles / sl["seconds"], 1), "unit": "evals/s", "seconds": round(sl["seconds"], 3),
                                "chunk_docs": args.e2e_stream, "report_bytes": sl["report_bytes"],
                                "report_GBps": round(sl["report_bytes"] / sl["seconds"] / 1e9, 3),
                                "exit_code": sl["exit_code"],
                                "note": "cfn_guard_validate_batch_stream_ex -o sarif in a process of its own: load + "
                                        "evaluation of every chunk (held on the device), then the SARIF frame and each "
                                        "chunk's device-rendered results to host memory"}
        except Exception as e:
            e2e_stream_sarif = {"value": None, "error": str(e)[-500:]}

    e2e_devices = None
    leg = None
    if (rank == 0 and not args.no_e2e and args.e2e_devices_docs and args.workload in ("cfg2", "cfg3")
            and args.loader == "device" and torch.cuda.device_count() >= world):
        # the in-library multi-GPU path (SURVEY.md 8(b) n_gpus): one process (rank 0, after the ranks' timed
        # region) drives devices 0 .. N-1 of an N-rank run, each device a pipeline of its own over chunks
        # k = d (mod N), the report written in document order (counted by the library's native callback);
        # weak scaling, --e2e-devices-docs per device.  One device: the one-device stream entry's chunks
        ndev = world
        nd = args.e2e_devices_docs * ndev
        dchunk = args.e2e_devices_chunk if ndev > 1 else args.e2e_stream
        if world == 1 and "devices" in early:
            leg = early["devices"]   # run before this process touched the GPU (above)
        else:
            log("e2e devices: %d documents over %d device(s), chunks of %d" % (nd, ndev, dchunk))
            try:
                leg = _stream_leg(args.workload, first, nd, args.resources, args.format, dchunk, ndev, threads)
            except Exception as e:
                leg = {"error": str(e)[-500:]}
    if leg is not None and "error" in leg:
        e2e_devices = {"value": None, "devices": ndev, "error": leg["error"]}
    elif leg is not None:
        t_dv, t_gen_d, dv_code = leg["seconds"], leg["gen_s"], leg["exit_code"]
        nb = [leg["report_bytes"]]
        e2e_devices = {"value": round(nd * nfiles / t_dv, 1), "unit": "evals/s", "devices": ndev, "docs": nd,
                       "docs_per_device": args.e2e_devices_docs, "chunk_docs": dchunk,
                       "seconds": round(t_dv, 3), "report_bytes": nb[0], "report_GBps": round(nb[0] / t_dv / 1e9, 3),
                       "exit_code": dv_code, "gen_s": round(t_gen_d, 3),
                       "note": "cfn_guard_validate_batch_stream_devices over devices 0..N-1 from one child process of rank 0 "
                               "(load + upload + evaluation + fetch + device-rendered JSON report to host memory, in "
                               "document order); text generation (gen_s) not included"}

    total_units = ntiles * world * args.steps
    value = total_units / elapsed
    if args.workload == "cfg5":
        workload = ("cfg5: %d AWS Config snapshots/GPU (%d configuration items) x %d-file network-reachability pack"
                    % (args.docs, n_ci * world, nfiles))
    elif args.workload == "cfg4":
        workload = ("cfg4: %d Terraform plans/GPU (%d resource_changes, 200-2000 per plan) x %d-file terraform pack"
                    % (args.docs, n_changes * world, nfiles))
    else:
        workload = "%s: %d synthetic CFN templates/GPU (%d resources) x %d-file rule pack" % (
            args.workload, args.docs, args.resources, nfiles)
        if args.format == "yaml":
            workload += " (block-style YAML text)"
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
                       "nodes": sess_stats["nodes"], "pool_bytes": sess_stats["pool_bytes"],
                       "tiles_fail_pass_skip_err": [n_fail, n_pass, n_skip, n_err],
                       "loader": args.loader, "load_s": round(t_load, 2), "host_threads": threads,
                       "upload_s": round(t_upload, 2), "device_loader": load_stats,
                       "rule_tallies_sum": tally_sum, "rule_tallies_fetched": int(sum(tally)),
                       "lane_tiles_retried_in_wave_mode": sess_stats["retried"],
                       "kernel_mode": sess_stats["mode"], "regex_memo": args.rx_memo,
                       "host": host_info()},
        }
        line["cpu_baseline"] = cpu
        if e2e is not None and e2e_stream is not None and e2e_stream.get("value"):
            # the headline end-to-end figure is one wall clock: the streamed C-ABI entry a caller uses; the
            # one-session phases timed one by one and summed stay beside it
            e2e["phase_sum_value"] = e2e["value"]
            e2e["value"] = e2e_stream["value"]
            e2e["value_source"] = "e2e_stream (one wall clock over load + evaluation + report, JSON)"
        line["e2e"] = e2e
        if e2e_sarif is not None:
            line["e2e_sarif"] = e2e_sarif
        if e2e_stream is not None:
            line["e2e_stream"] = e2e_stream
        if e2e_stream_sarif is not None:
            line["e2e_stream_sarif"] = e2e_stream_sarif
        if e2e_devices is not None:
            line["e2e_stream_devices"] = e2e_devices
        if gather is not None:
            line["report_gather"] = gather
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
