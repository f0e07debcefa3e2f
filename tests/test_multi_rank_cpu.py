"""World-size-2 sharding + tally reduction on CPU (gloo): the N>1 path of bench.py.

Each rank evaluates its shard of the synthetic corpus with the CPU oracle (standing in for the
device statuses, which need a GPU), fills the same tally layout rule_count_kernel writes, and
all-reduces it; rank 0 checks the sum against a single-process evaluation of both shards."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import sharding  # noqa: E402
import synth  # noqa: E402

DOCS_PER_RANK = 3
RULES = [("iam.guard", synth.IAM_RULES), ("ebs.guard", synth.EBS_RULES)]


def _tallies(first, n):
    from guard_oracle.parser import parse_rules
    from guard_oracle.loader import load_document
    from guard_oracle import evaluator as E
    parsed = [parse_rules(t, name) for name, t in RULES]
    max_top = max(len(rf["guard_rules"]) for rf in parsed)
    code = {"PASS": 0, "FAIL": 1, "SKIP": 2}
    out = torch.zeros(sharding.tally_size(len(parsed), max_top), dtype=torch.int64)
    for i, text in enumerate(synth.cfn_corpus(n, start=first, n_resources=12)):
        doc = load_document(text, "d%d" % (first + i))
        for f, rf in enumerate(parsed):
            root = E.RootScope(rf, doc)
            status = E.eval_rules_file(rf, root, "d")
            out[sharding.tally_index(f, max_top, code[status], max_top)] += 1
    return out


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = sharding.shard_range(rank, world, DOCS_PER_RANK)
    t = sharding.all_reduce_tallies(_tallies(first, n), dist)
    if rank == 0:
        q.put(t.tolist())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_ranges_partition_the_corpus():
    got = [sharding.shard_range(r, 4, 10) for r in range(4)]
    assert got == [(0, 10), (10, 10), (20, 10), (30, 10)]
    with pytest.raises(ValueError):
        sharding.shard_range(4, 4, 10)


def test_two_rank_tally_reduction_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    reduced = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert reduced == _tallies(0, 2 * DOCS_PER_RANK).tolist()
    assert sum(reduced) == 2 * DOCS_PER_RANK * len(RULES)


# ---- failure-record / report gather to rank 0 ----
REPORT_DOCS = 3


def _shard_report(first, n, output):
    from guard_oracle import validate_structured
    docs = [("synthetic-%d.json" % (first + i), t)
            for i, t in enumerate(synth.cfn_corpus(n, start=first, n_resources=10))]
    text, code, _ = validate_structured(RULES, docs, output=output)
    return text, code


def _report_worker(rank, world, port, q, codes):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for fmt in ("json", "yaml", "sarif", "junit"):
        first, n = sharding.shard_range(rank, world, REPORT_DOCS)
        text, code = _shard_report(first, n, fmt)
        out[fmt] = sharding.gather_report(text, code, dist, output=fmt)
    # exit-code precedence with a different code on every rank
    out["codes"] = [sharding.reduce_exit_code(c[rank], dist) for c in codes]
    if rank == 0:
        q.put(out)
    else:
        assert all(out[f][0] is None for f in ("json", "yaml", "sarif", "junit"))
    dist.destroy_process_group()


def test_two_rank_report_gather_matches_single_process():
    codes = [(0, 19), (5, 19), (19, 5), (0, 5), (0, 0), (-1, 19), (5, -1)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_report_worker, args=(r, 2, port, q, codes)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for fmt in ("json", "yaml", "sarif", "junit"):
        full, code = _shard_report(0, 2 * REPORT_DOCS, fmt)
        assert got[fmt] == (full, code), fmt
    assert got["codes"] == [19, 19, 19, 5, 0, -1, -1]


def test_merge_reports_edge_cases():
    assert sharding.merge_reports(["[]", "[]"]) == "[]"
    assert sharding.merge_reports(["[]\n"], "yaml") == "[]\n"
    assert sharding.merge_reports(["[\n  1\n]", "[]", "[\n  2\n]"]) == "[\n  1,\n  2\n]"
    with pytest.raises(ValueError):
        sharding.merge_reports(["{}"])
    with pytest.raises(ValueError):
        sharding.merge_reports(["x"], "junit")


def test_byte_balanced_shard_ranges():
    sizes = [10, 10, 10, 70, 5, 5, 5, 5, 40, 40]
    r = sharding.shard_ranges_by_bytes(sizes, 3)
    assert [c for _, c in r] and sum(c for _, c in r) == len(sizes)
    assert all(r[i][0] + r[i][1] == r[i + 1][0] for i in range(2))   # contiguous, in order
    loads = [sum(sizes[a:a + n]) for a, n in r]
    assert max(loads) <= 100 and min(c for _, c in r) >= 1
    assert sharding.shard_ranges_by_bytes([1] * 8, 4) == [(0, 2), (2, 2), (4, 2), (6, 2)]
    assert sharding.shard_ranges_by_bytes([5], 2) == [(0, 0), (0, 1)]   # fewer documents than ranks


# ---- streamed gather in bounded blocks (sharding.stream_report) ----
STREAM_DOCS = 4


def _stream_worker(rank, world, port, q, fail_at):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import io
    out = {}
    for fmt in ("json", "yaml", "sarif", "junit"):
        first, n = sharding.shard_range(rank, world, STREAM_DOCS)
        _, code = _shard_report(first, n, fmt)

        def render(f, c, first=first, fmt=fmt):
            if fail_at is not None and rank == fail_at[0] and f == fail_at[1]:
                raise RuntimeError("report of document %d aborted" % (first + f))
            return _shard_report(first + f, c, fmt)[0]
        sink = io.StringIO()
        # blocks of one document: every block is smaller than one rank's report
        res = sharding.stream_report(render, n, code, dist, sink, output=fmt, block_docs=1, lookahead=2)
        out[fmt] = (sink.getvalue() if rank == 0 else None, res)
        if fmt in ("json", "yaml") and fail_at is None:
            # the bulk path: bytes blocks in, memoryview pieces out (no decode per block)
            bsink = io.BytesIO()
            res = sharding.stream_report(lambda f, c: render(f, c).encode(), n, code, dist, bsink, output=fmt,
                                         block_docs=2, raw=True)
            out[fmt + "_raw"] = (bsink.getvalue().decode() if rank == 0 else None, res)
    q.put((rank, out))
    dist.destroy_process_group()


def _run_stream(fail_at=None, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, q, fail_at)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_streamed_report_in_one_document_blocks_matches_single_process():
    got = _run_stream()
    for fmt in ("json", "yaml", "sarif", "junit", "json_raw", "yaml_raw"):
        full, code = _shard_report(0, 2 * STREAM_DOCS, fmt.split("_")[0])
        text, res = got[0][fmt]
        assert res == (code, None), fmt
        assert text == full, fmt
        assert got[1][fmt] == (None, (code, None)), fmt


def test_streamed_report_error_ends_the_stream_on_every_rank():
    got = _run_stream(fail_at=(1, 2))   # rank 1's third block aborts
    for fmt in ("json", "yaml", "sarif", "junit"):
        for r in (0, 1):
            code, msg = got[r][fmt][1]
            assert code == -1, (fmt, r)
        assert got[0][fmt][1][1] == "report of document %d aborted" % (STREAM_DOCS + 2)


def test_report_merger_sarif_and_junit_edges():
    full, _ = _shard_report(0, 3, "sarif")
    # three shards, the middle one with no documents: artifacts de-duplicated and in order
    parts = [_shard_report(0, 1, "sarif")[0], _shard_report(1, 0, "sarif")[0], _shard_report(1, 2, "sarif")[0]]
    assert sharding.merge_reports(parts, "sarif") == full
    j = [_shard_report(0, 0, "junit")[0], _shard_report(0, 3, "junit")[0]]
    assert sharding.merge_reports(j, "junit") == _shard_report(0, 3, "junit")[0]
    with pytest.raises(ValueError):
        sharding.merge_reports(["{}"], "sarif")
