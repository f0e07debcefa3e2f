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


def shard_ranges_by_bytes(sizes, world):
    """Contiguous document ranges [(first, count)] per rank, balanced by document bytes (the arena a
    document becomes is proportional to its text).  Contiguity keeps rank order =
    document order, so gathered reports stitch into the single-process output."""
    total = sum(sizes)
    out, start, acc = [], 0, 0
    for r in range(world):
        target = total * (r + 1) / world
        end = start
        while end < len(sizes) and (acc + sizes[end] <= target or end == start) and len(sizes) - end > world - r - 1:
            acc += sizes[end]
            end += 1
        if r == world - 1:
            while end < len(sizes):
                acc += sizes[end]
                end += 1
        out.append((start, end - start))
        start = end
    return out


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
# the per-rank texts are gathered to rank 0 (all_gather of the byte counts, then point-to-point
# send / recv of each rank's bytes to rank 0 only: RCCL on GPU ranks, gloo on CPU) and stitched in
# rank order.  Rank order is document order, so the result is the single-process
# `validate --structured` output (reporters/validate/structured.rs:99-133 writes one FileReport per
# data file, in input order); SARIF and JUnit runs are re-totalled (sarif.rs, xml.rs).

# exit-code precedence of a structured run (commands/validate.rs:391-403, structured.rs:111-113):
# an evaluation error aborts the run (-1); otherwise any FAIL sets 19, which overrides the
# rules-file parse error code 5; 0 when everything passed or skipped.
_SEVERITY = {0: 0, 5: 1, 19: 2, -1: 3}
_BY_SEVERITY = {v: k for k, v in _SEVERITY.items()}


def collective_device(dist, device=None):
    """The device a collective's tensors live on: the caller's choice, else the current GPU under
    the nccl (RCCL) backend -- which accepts device tensors only -- and the CPU under gloo."""
    import torch
    if device is not None:
        return torch.device(device)
    if dist is not None and dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def reduce_exit_code(code, dist, device=None):
    """The job's exit code from every rank's (all_reduce MAX over the precedence above)."""
    import torch
    if code not in _SEVERITY:
        raise ValueError("unknown structured exit code %r" % (code,))
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return code
    device = collective_device(dist, device)
    t = torch.tensor([_SEVERITY[code]], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return _BY_SEVERITY[int(t.item())]


def gather_bytes(payload, dist, device=None):
    """Every rank's `payload` (bytes) in rank order on rank 0; None on the other ranks.  The byte
    counts are all-gathered (8 B per rank); then each rank sends its bytes to rank 0 alone, so a
    rank holds only its own report and rank 0 the job's (no world-sized padded buffers).  Under
    RCCL the buffers are device tensors (collective_device); under gloo host tensors."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [payload]
    device = collective_device(dist, device)
    world, rank = dist.get_world_size(), dist.get_rank()
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if rank != 0:
        if sizes[rank]:
            buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
            dist.send(buf, dst=0)
        return None
    parts = [payload]
    for r in range(1, world):
        if not sizes[r]:
            parts.append(b"")
            continue
        buf = torch.empty(sizes[r], dtype=torch.uint8, device=device)
        dist.recv(buf, src=r)
        parts.append(bytes(buf.cpu().numpy().tobytes()))
    return parts


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
    if output == "sarif":
        return _merge_sarif(parts)
    if output == "junit":
        return _merge_junit(parts)
    raise ValueError("unknown output format %r" % (output,))


def _merge_sarif(parts):
    """SarifReport (reporters/validate/sarif.rs): one run whose artifacts are the distinct failing
    data files in order and whose results are every failure in order; serde_json pretty text."""
    import json
    from collections import OrderedDict
    docs = [json.loads(p, object_pairs_hook=OrderedDict) for p in parts]
    base = docs[0]
    run = base["runs"][0]
    seen = {json.dumps(a, sort_keys=True) for a in run["artifacts"]}
    for d in docs[1:]:
        r = d["runs"][0]
        for a in r["artifacts"]:
            k = json.dumps(a, sort_keys=True)
            if k not in seen:
                seen.add(k)
                run["artifacts"].append(a)
        run["results"].extend(r["results"])
    return json.dumps(base, indent=2, ensure_ascii=False)


def _merge_junit(parts):
    """JunitReport (reporters/validate/xml.rs): the test suites in order under one <testsuites> whose
    tests / failures / errors are the sums."""
    import re
    head = re.compile(r'^(<\?xml[^\n]*\n)<testsuites name="([^"]*)" tests="(\d+)" failures="(\d+)" errors="(\d+)" time="([^"]*)">\n')
    tests = failures = errors = 0
    bodies = []
    decl = name = time = None
    for p in parts:
        m = head.match(p)
        if not m or not p.endswith("</testsuites>\n"):
            raise ValueError("not a JUnit report")
        decl, name, time = m.group(1), m.group(2), m.group(6)
        tests += int(m.group(3))
        failures += int(m.group(4))
        errors += int(m.group(5))
        bodies.append(p[m.end():-len("</testsuites>\n")])
    return '%s<testsuites name="%s" tests="%d" failures="%d" errors="%d" time="%s">\n%s</testsuites>\n' % (
        decl, name, tests, failures, errors, time, "".join(bodies))


def gather_report(local_text, local_code, dist, output="json", device=None):
    """Rank 0: (merged structured report, job exit code); other ranks: (None, job exit code)."""
    code = reduce_exit_code(local_code, dist, device)
    parts = gather_bytes(local_text.encode(), dist, device)
    if parts is None:
        return None, code
    return merge_reports([p.decode() for p in parts], output), code
