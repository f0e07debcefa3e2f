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
