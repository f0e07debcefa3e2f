"""One rank of the two-rank GPU rehearsal in tests/test_gpu_multi_rank.py (not collected by pytest).

Started as a child process (subprocess) before it touches the GPU; joins a gloo group (RANK /
WORLD_SIZE / MASTER_* from the environment), evaluates its byte-balanced shard of the corpus on
device 0 through the C ABI, all-reduces the device tallies and streams its structured reports to rank 0
(sharding.stream_report, blocks of 7 documents), which writes them and the reduced tallies under argv[1]."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "cloudformation-guard_amd"))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import guard_amd  # noqa: E402
import sharding  # noqa: E402
import synth  # noqa: E402
from rulepack import rule_pack  # noqa: E402

N_DOCS = 150


def main():
    out = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    docs = synth.cfn_corpus(N_DOCS, start=321)
    first, count = sharding.shard_ranges_by_bytes([len(d) for d in docs], world)[rank]
    s = guard_amd.Session()
    for name, text in rule_pack("cfg2"):
        s.add_rules(text, name)
    s.add_docs(docs[first:first + count], ["synthetic-%d.json" % (first + i) for i in range(count)])
    s.eval(1)
    tallies = torch.tensor(s.counts(), dtype=torch.int64)
    sharding.all_reduce_tallies(tallies, dist)
    res = {"tallies": tallies.tolist(), "codes": {}}
    for fmt in ("json", "yaml", "sarif", "junit"):
        sink = open(os.path.join(out, "report." + fmt), "w") if rank == 0 else None
        code, err = sharding.stream_report(lambda f, c, fmt=fmt: s.report_range(fmt, f, c)[0], count,
                                           s.exit_code(fmt), dist, sink, output=fmt, block_docs=7)
        if sink:
            sink.close()
        res["codes"][fmt] = [code, err]
    if rank == 0:
        with open(os.path.join(out, "result.json"), "w") as f:
            json.dump(res, f)
    s.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
