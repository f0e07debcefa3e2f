"""Document sharding and tally reduction for N ranks.

Documents shard with no data-path exchange: rank r owns templates [r*D, (r+1)*D) (weak scaling,
D per GPU).  The only collective is the all-reduce of the per-(rules file, rule) PASS/FAIL/SKIP/
error tallies that rule_count_kernel writes (layout in include/cfn_guard_mi355x.h).
"""

import io
import queue
import re
import threading

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
# The structured report of a sharded run: every rank reports its own documents in
# bounded blocks and sends them point-to-point to rank 0 (RCCL on GPU ranks, gloo on CPU), which joins
# them in rank order as they arrive (stream_report / ReportMerger).  Rank order is document order, so the
# result is the single-process `validate --structured` output; SARIF runs and JUnit suites are
# re-totalled from the blocks' text, without parsing whole reports.

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


class ReportMerger:
    """Rank 0's incremental join of per-shard structured report blocks into the single-process
    `validate --structured` text (reporters/validate/structured.rs:99-133 writes one FileReport per data
    file, in input order; sarif.rs one run; xml.rs one <testsuites>), written to `sink` (a .write(str)
    object) as blocks arrive -- it holds one block at a time, plus SARIF's distinct artifact entries.

    Blocks are the texts a writer over a contiguous document range produces (gg_session_report_range),
    fed in document order.  json: serde_json pretty Vec<FileReport> -- "[]" when empty, else "[\n" items
    joined by ",\n" "\n]"; yaml: a top-level block sequence -- "[]\n" when empty, else "- " items back to
    back.  sarif and junit take two passes over the blocks ("head" then "body"): the artifact list (distinct
    failing files, in order) / the suite totals precede the results / suites in the output."""

    PHASES = {"json": ("body",), "yaml": ("body",), "sarif": ("head", "body"), "junit": ("head", "body")}
    _SARIF_ART = '\n      "artifacts": '
    _SARIF_RES = '\n      "results": '
    _JUNIT_HEAD = re.compile(r'^(<\?xml[^\n]*\n)<testsuites name="([^"]*)" tests="(\d+)" failures="(\d+)" '
                             r'errors="(\d+)" time="([^"]*)">\n')

    def __init__(self, output, sink):
        if output not in self.PHASES:
            raise ValueError("unknown output format %r" % (output,))
        self.output, self.sink = output, sink
        self.items = 0
        self.head = None          # sarif: text up to '"artifacts": '; junit: (decl, name, time)
        self.tail = None          # sarif: text after the results array
        self.arts, self.seen = [], set()
        self.totals = [0, 0, 0]

    # ---- sarif text layout (serde_json pretty, 2-space indent: run members at indent 6, their items at 8)
    def _sarif_split(self, text):
        a = text.find(self._SARIF_ART)
        r = text.find(self._SARIF_RES)
        if a < 0 or r < a or not text.startswith("{\n"):
            raise ValueError("not a SARIF report")
        head = text[:a + len(self._SARIF_ART)]
        arts = text[a + len(self._SARIF_ART):r - 1]       # the array, without the "," before "results"
        rest = text[r + len(self._SARIF_RES):]
        if rest.startswith("[]"):
            results, tail = "", rest[2:]
        else:
            end = rest.find("\n      ]")
            if not rest.startswith("[\n") or end < 0:
                raise ValueError("not a SARIF report")
            results, tail = rest[2:end], rest[end + len("\n      ]"):]
        return head, arts, results, tail

    def _sarif_entries(self, arts):
        if arts == "[]":
            return []
        if not (arts.startswith("[\n") and arts.endswith("\n      ]")):
            raise ValueError("not a SARIF artifact list")
        # items sit at indent 8 and their members deeper, so "},\n        {" only separates items
        return re.split(r"(?<=\n        \}),\n(?=        \{)", arts[2:-len("\n      ]")])

    def feed(self, phase, text):
        """one block: a str, or for json / yaml a bytes-like block (raw=True: UTF-8 bytes, written as
        memoryview slices without a decode or a copy)"""
        out = self.output
        raw = not isinstance(text, str)
        if raw and out in ("sarif", "junit"):
            text = bytes(text).decode()
            raw = False
        if raw:
            text = memoryview(text).cast("B")
        lit = (lambda x: x.encode()) if raw else (lambda x: x)
        if out == "json":
            if len(text) == 2 and bytes(text) == b"[]" if raw else text == "[]":
                return
            if not (bytes(text[:2]) == b"[\n" and bytes(text[-2:]) == b"\n]" if raw
                    else text.startswith("[\n") and text.endswith("\n]")):
                raise ValueError("not a pretty JSON array of file reports")
            self.sink.write(lit("[\n" if self.items == 0 else ",\n"))
            self.sink.write(text[2:-2])
            self.items += 1
        elif out == "yaml":
            if (bytes(text) == b"[]\n" if raw and len(text) == 3 else (not raw and text == "[]\n")):
                return
            if not (bytes(text[:2]) == b"- " if raw else text.startswith("- ")):
                raise ValueError("not a YAML sequence of file reports")
            self.sink.write(text)
            self.items += 1
        elif out == "sarif":
            head, arts, results, tail = self._sarif_split(text)
            if phase == "head":
                if self.head is None:
                    self.head, self.tail = head, tail
                for e in self._sarif_entries(arts):
                    if e not in self.seen:
                        self.seen.add(e)
                        self.arts.append(e)
                return
            if self.items == 0:
                self._sarif_open()
            if results:
                self.sink.write("[\n" if self.items == 1 else ",\n")
                self.sink.write(results)
                self.items += 1
        else:
            m = self._JUNIT_HEAD.match(text)
            if not m or not text.endswith("</testsuites>\n"):
                raise ValueError("not a JUnit report")
            if phase == "head":
                if self.head is None:
                    self.head = (m.group(1), m.group(2), m.group(6))
                for k in range(3):
                    self.totals[k] += int(m.group(3 + k))
                return
            if self.items == 0:
                decl, name, time_ = self.head
                self.sink.write('%s<testsuites name="%s" tests="%d" failures="%d" errors="%d" time="%s">\n'
                                % (decl, name, self.totals[0], self.totals[1], self.totals[2], time_))
                self.items = 1
            self.sink.write(text[m.end():-len("</testsuites>\n")])

    def _sarif_open(self):
        self.sink.write(self.head)
        if self.arts:
            self.sink.write("[\n" + ",\n".join(self.arts) + "\n      ]")
        else:
            self.sink.write("[]")
        self.sink.write("," + self._SARIF_RES)
        self.items = 1          # 1: results not opened yet; > 1: results written

    def finish(self, raw=False):
        out = self.output
        lit = (lambda x: x.encode()) if raw else (lambda x: x)
        if out == "json":
            self.sink.write(lit("\n]" if self.items else "[]"))
        elif out == "yaml":
            if not self.items:
                self.sink.write(lit("[]\n"))
        elif out == "sarif":
            if self.head is None:
                raise ValueError("no SARIF blocks")
            if self.items == 0:
                self._sarif_open()
            self.sink.write("[]" if self.items == 1 else "\n      ]")
            self.sink.write(self.tail)
        else:
            if self.head is None:
                raise ValueError("no JUnit blocks")
            if self.items == 0:
                self.feed("body", "%s<testsuites name=\"%s\" tests=\"0\" failures=\"0\" errors=\"0\" time=\"%s\">\n"
                          "</testsuites>\n" % (self.head[0], self.head[1], self.head[2]))
            self.sink.write("</testsuites>\n")


def merge_reports(parts, output="json"):
    """Stitch whole per-shard structured reports (document order) into the single-process output --
    ReportMerger over one block per shard."""
    out = io.StringIO()
    m = ReportMerger(output, out)
    for phase in ReportMerger.PHASES[output]:
        for p in parts:
            m.feed(phase, p)
    m.finish()
    return out.getvalue()


def _blocks(render, ndocs, block_docs, lookahead, stage=None, stage_bytes=0):
    """render(first, count) over [0, ndocs) in blocks on a thread (the library releases the GIL), at most
    `lookahead` blocks ahead -- or, with stage(block) -> staged copy (a device tensor in HBM) and a byte
    budget stage_bytes, as many blocks as fit the budget, so a rank renders its whole report while rank 0
    is still busy with earlier ranks; yields ("ok", block) then, on a render error, ("error", message)"""
    q = queue.Queue()
    stop = threading.Event()
    cv = threading.Condition()
    held = [0, 0]       # blocks, bytes queued and not yet consumed

    def room(nbytes):
        if stage_bytes:
            return held[1] == 0 or held[1] + nbytes <= stage_bytes
        return held[0] < max(1, lookahead)

    def work():
        try:
            starts = list(range(0, ndocs, block_docs)) or [0]
            last = 0
            for f in starts:
                with cv:
                    while not stop.is_set() and not room(last):
                        cv.wait(0.1)
                if stop.is_set():
                    return
                b = render(f, min(block_docs, ndocs - f))
                if stage is not None:
                    b = stage(b)
                last = len(b)
                with cv:
                    held[0] += 1
                    held[1] += last
                q.put(("ok", b))
            q.put(None)
        except Exception as e:     # a report that aborts (GuardError): its message ends the stream
            q.put(("error", "%s" % (e,)))
            q.put(None)

    th = threading.Thread(target=work, daemon=True)
    th.start()
    try:
        while True:
            item = q.get()
            if item is None:
                return
            yield item
            if item[0] == "error":
                return
            with cv:
                held[0] -= 1
                held[1] -= len(item[1])
                cv.notify()
    finally:
        stop.set()
        with cv:
            cv.notify()
        th.join()


_END, _ERROR = -1, -2


def _as_u8(payload):
    """a uint8 torch tensor over a block's bytes (str: UTF-8 encoded; bytes-like / numpy: no copy)"""
    import numpy as np
    import torch
    if isinstance(payload, str):
        payload = payload.encode()
    a = payload if isinstance(payload, np.ndarray) else np.frombuffer(payload, dtype=np.uint8)
    if not a.flags.writeable:
        a = a.copy()
    return torch.from_numpy(a)


def _send_msg(kind_or_len, payload, dist, device, dst=0):
    import torch
    dist.send(torch.tensor([kind_or_len], dtype=torch.int64, device=device), dst=dst)
    if payload is not None and len(payload):
        buf = payload if isinstance(payload, torch.Tensor) else _as_u8(payload)
        if buf.device != device:
            buf = buf.to(device)
        dist.send(buf, dst=dst)


class _Landing:
    """rank 0's receive buffers, reused across blocks: a device buffer (RCCL) and a pinned host copy"""

    def __init__(self, device):
        self.device, self.dev, self.host = device, None, None

    def get(self, n):
        import torch
        if self.dev is None or self.dev.numel() < n:
            self.dev = torch.empty(max(n, 1 << 20), dtype=torch.uint8, device=self.device)
            if self.device.type != "cpu":
                self.host = torch.empty(self.dev.numel(), dtype=torch.uint8).pin_memory()
        return self.dev[:n]

    def to_host(self, buf, n):
        if self.device.type == "cpu":
            return buf.numpy()
        self.host[:n].copy_(buf)
        return self.host[:n].numpy()


def _recv_msg(src, dist, device, landing, raw):
    """(length or _END / _ERROR, payload: str, or with raw a uint8 numpy view valid until the next receive)"""
    import torch
    n = torch.zeros(1, dtype=torch.int64, device=device)
    dist.recv(n, src=src)
    n = int(n.item())
    ln = n if n >= 0 else 0
    if n == _ERROR:
        m = torch.zeros(1, dtype=torch.int64, device=device)
        dist.recv(m, src=src)
        ln = int(m.item())
    if ln <= 0:
        return n, (b"" if raw and n != _ERROR else "")
    buf = landing.get(ln)
    dist.recv(buf, src=src)
    host = landing.to_host(buf, ln)
    if raw and n != _ERROR:
        return n, host
    return n, host.tobytes().decode()


def stream_report(render, ndocs, local_code, dist, sink=None, output="json", block_docs=4096, lookahead=2,
                  device=None, raw=False, stage_bytes=None):
    """The structured report of a sharded job, streamed to rank 0's `sink` in bounded chunks.

    Every rank renders its own documents in blocks of `block_docs` (render(first, count) -> text, e.g.
    Session.report_range; `lookahead` blocks ahead on a thread) and sends them to rank 0 one block at a
    time (the length, then the bytes: RCCL device buffers under nccl, host tensors under gloo); rank 0 joins
    them in rank order -- document order -- with ReportMerger as they arrive.  Memory is one block per rank
    in flight (rank 0: one block at a time), whatever the report's size; sarif / junit take two passes.

    Returns (job exit code, error message or None) on every rank: the exit code reduced over the ranks'
    local codes (-1 > 19 > 5 > 0); an evaluation error anywhere (-1) streams nothing; a report that aborts
    while rendering ends the stream with the first such error in document order, code -1.

    raw=True: render returns bytes-like blocks (Session.report_range_raw: the library's buffer, no copy)
    and rank 0's sink receives bytes-like pieces (json / yaml: memoryview slices of the landing buffers,
    valid during the write call) -- the bulk path, with no UTF-8 decode or Python string per block.  Under
    RCCL a sending rank stages its rendered blocks in its own HBM (up to stage_bytes; None: 80 % of the
    device's free memory), so every rank renders its whole report concurrently and rank 0's receive is
    bounded by xGMI and its own device-to-host copy, not by the other ranks' rendering."""
    code = reduce_exit_code(local_code, dist, device)
    if code == -1:
        return -1, None
    multi = dist is not None and dist.is_initialized() and dist.get_world_size() > 1
    world, rank = (dist.get_world_size(), dist.get_rank()) if multi else (1, 0)
    device = collective_device(dist, device) if multi else None
    merger = ReportMerger(output, sink) if rank == 0 else None
    landing = _Landing(device) if multi and rank == 0 else None
    error = None
    for phase in ReportMerger.PHASES[output]:
        if rank != 0:
            failed = False
            stage, budget = None, 0
            if device.type != "cpu":
                import torch
                budget = int(0.8 * torch.cuda.mem_get_info(device)[0]) if stage_bytes is None else int(stage_bytes)
                if budget > 0:
                    stage = lambda b: _as_u8(b).to(device)   # noqa: E731  (H2D on the render thread)
            for kind, text in _blocks(render, ndocs, block_docs, lookahead, stage, budget):
                b = text.encode() if isinstance(text, str) else text
                if kind == "error":
                    _send_msg(_ERROR, None, dist, device)
                    _send_msg(len(b), b, dist, device)
                    failed = True
                    break
                _send_msg(len(b), b, dist, device)
            if not failed:
                _send_msg(_END, None, dist, device)
            continue
        for r in range(world):
            if r == 0:
                for kind, text in _blocks(render, ndocs, block_docs, lookahead):
                    if kind == "error":
                        error = error or text
                        break
                    if error is None:
                        merger.feed(phase, text)
                continue
            while True:
                n, payload = _recv_msg(r, dist, device, landing, raw)
                if n == _END:
                    break
                if n == _ERROR:
                    error = error or payload
                    break
                if error is None:
                    merger.feed(phase, payload)
    if rank == 0 and error is None:
        merger.finish(raw=raw)
    if multi:
        import torch
        flag = torch.tensor([1 if error is not None else 0], dtype=torch.int64, device=device)
        dist.broadcast(flag, src=0)
        if int(flag.item()):
            return -1, error
    return (-1, error) if error is not None else (code, None)


def gather_report(local_text, local_code, dist, output="json", device=None):
    """Rank 0: (merged structured report, job exit code); other ranks: (None, job exit code).  Each rank's
    whole text is one block of stream_report (rank 0 collects the stream in memory: small reports and tests;
    stream_report with a file sink is the bounded-memory path)."""
    out = io.StringIO()
    code, err = stream_report(lambda f, c: local_text, 1, local_code, dist, out, output, block_docs=1, device=device)
    if err is not None:
        raise RuntimeError(err)
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    return (out.getvalue() if rank == 0 and code != -1 else None), code
