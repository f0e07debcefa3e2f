"""Document sharding and tally reduction for N ranks.

Documents shard with no data-path exchange: rank r owns templates [r*D, (r+1)*D) (weak scaling,
D per GPU).  The only collective is the all-reduce of the per-(rules file, rule) PASS/FAIL/SKIP/
error tallies that rule_count_kernel writes (layout in include/cfn_guard_mi355x.h).
"""

STATUSES = ("PASS", "FAIL", "SKIP", "ERROR")


def shard_range(rank, world, docs_per_rank):
    """Templates owned by `rank` under weak scaling."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return rank * docs_per_rank, docs_per_rank


def tally_index(file, rule, status, max_top):
    """Index into the tally vector: ((file * (max_top + 1) + rule) * 4) + status.
    rule == max_top is the file-level line (file status, errored tiles in status 3)."""
    return (file * (max_top + 1) + rule) * 4 + status


def tally_size(nfiles, max_top):
    return nfiles * (max_top + 1) * 4


def all_reduce_tallies(tensor, dist):
    """Sum the tally tensor across ranks (RCCL on GPU ranks, gloo in the CPU tests)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tensor)
    return tensor


# ---------------------------------------------------------------- reports -----
# The structured report of a sharded run: every rank reports its own documents;
# the per-rank texts are gathered to rank 0 (all_gather of the byte counts, then one padded
# all_gather of the bytes: RCCL on GPU ranks, gloo on CPU) and stitched in rank order.  Rank order
# is document order, so the result is the single-process `validate --structured` output
# (reporters/validate/structured.rs:99-133 writes one FileReport per data file, in input order).

# exit-code precedence of a structured run (commands/validate.rs:391-403, structured.rs:111-113):
# an evaluation error aborts the run (-1); otherwise any FAIL sets 19, which overrides the
# rules-file parse error code 5; 0 when everything passed or skipped.
_SEVERITY = {0: 0, 5: 1, 19: 2, -1: 3}
_BY_SEVERITY = {v: k for k, v in _SEVERITY.items()}


def reduce_exit_code(code, dist, device="cpu"):
    """The job's exit code from every rank's (all_reduce MAX over the precedence above)."""
    import torch
    if code not in _SEVERITY:
        raise ValueError("unknown structured exit code %r" % (code,))
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return code
    t = torch.tensor([_SEVERITY[code]], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return _BY_SEVERITY[int(t.item())]


def gather_bytes(payload, dist, device="cpu"):
    """Every rank's `payload` (bytes) in rank order on rank 0; None on the other ranks."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [payload]
    world = dist.get_world_size()
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    cap = max(1, max(sizes))
    buf = torch.zeros(cap, dtype=torch.uint8, device=device)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    parts = [torch.empty(cap, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(parts, buf)
    if dist.get_rank() != 0:
        return None
    return [bytes(p[:s].cpu().numpy().tobytes()) for p, s in zip(parts, sizes)]


def merge_reports(parts, output="json"):
    """Stitch per-shard structured reports (rank order) into the single-process output.

    json: serde_json::to_writer_pretty of Vec<FileReport> -- "[]" when empty, else "[\\n" items
    joined by ",\\n" "\\n]"; yaml: serde_yaml of a top-level sequence -- "[]\\n" when empty, else
    the "- " items back to back."""
    if output == "json":
        bodies = []
        for p in parts:
            if p == "[]":
                continue
            if not (p.startswith("[\n") and p.endswith("\n]")):
                raise ValueError("not a pretty JSON array of file reports")
            bodies.append(p[2:-2])
        return "[\n" + ",\n".join(bodies) + "\n]" if bodies else "[]"
    if output == "yaml":
        bodies = [p for p in parts if p != "[]\n"]
        for p in bodies:
            if not p.startswith("- "):
                raise ValueError("not a YAML sequence of file reports")
        return "".join(bodies) if bodies else "[]\n"
    raise ValueError("merge_reports supports json and yaml (SARIF / JUnit carry run-level totals)")


def gather_report(local_text, local_code, dist, output="json", device="cpu"):
    """Rank 0: (merged structured report, job exit code); other ranks: (None, job exit code)."""
    code = reduce_exit_code(local_code, dist, device)
    parts = gather_bytes(local_text.encode(), dist, device)
    if parts is None:
        return None, code
    return merge_reports([p.decode() for p in parts], output), code
