"""The N > 1 path on the GPU: two ranks (gloo, both on device 0, started as child processes before they
touch the GPU) each evaluate a byte-balanced shard through the C ABI, all-reduce the device tallies and
stream their structured reports to rank 0 in 7-document blocks (sharding.stream_report).  The reduced
tallies and the joined reports (all four formats, exit codes) must equal one process evaluating the whole
corpus.  This is the multi-rank evidence with the HIP kernel in the loop (the CPU test of the same
protocol, tests/test_multi_rank_cpu.py, uses oracle statuses)."""
import json
import os
import socket
import subprocess
import sys

import pytest

import guard_amd
import synth
from rulepack import rule_pack

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gpu_tallies_and_streamed_reports(tmp_path):
    sys.path.insert(0, HERE)
    import multi_rank_gpu_child as child
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GG_DEVICE="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "multi_rank_gpu_child.py"), str(tmp_path)],
                                      env=env))
    for p in procs:
        assert p.wait(timeout=180) == 0
    res = json.load(open(tmp_path / "result.json"))
    docs = synth.cfn_corpus(child.N_DOCS, start=321)
    s = guard_amd.Session()
    for name, text in rule_pack("cfg2"):
        s.add_rules(text, name)
    s.add_docs(docs, ["synthetic-%d.json" % i for i in range(len(docs))])
    s.eval(1)
    assert res["tallies"] == s.counts()
    assert sum(res["tallies"]) > 0
    for fmt in ("json", "yaml", "sarif", "junit"):
        text, code = s.report(fmt)
        assert res["codes"][fmt] == [code, None], fmt
        assert open(tmp_path / ("report." + fmt)).read() == text, fmt
    s.close()
