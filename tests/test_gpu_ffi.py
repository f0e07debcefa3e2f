"""guard-ffi drop-in under the call pattern of its users (guard-lambda, the fuzzers: one document x
one rules file per call, repeatedly, possibly from several threads; SURVEY.md 8(b) "Threading"):
results equal the oracle's run_checks, device state is reused across calls (DeviceBufs pool in
capi.cpp), and concurrent callers do not interfere.  Per-call latency is written to
gpurun_out/ffi_latency.json for DESIGN.md."""
import json
import os
import threading
import time

import pytest

import guard_amd
import synth
from guard_oracle import run_checks as oracle_run_checks
from rulepack import rule_pack

pytestmark = pytest.mark.gpu


def _cases(n):
    docs = synth.cfn_corpus(n, start=777, n_resources=8)
    rules = rule_pack()
    out = []
    for i, d in enumerate(docs):
        name, text = rules[i % len(rules)]
        out.append((d, "doc%d.json" % i, text, name, oracle_run_checks(d, "doc%d.json" % i, text, name)))
    return out


def test_sequential_calls_match_oracle_and_reuse_state():
    cases = _cases(48)
    guard_amd.run_checks(*cases[0][:4])   # first call: device init, pool fill
    lat = []
    for rep in range(3):
        for d, dn, r, rn, exp in cases:
            t = time.perf_counter()
            got = guard_amd.run_checks(d, dn, r, rn)
            lat.append(time.perf_counter() - t)
            assert got == exp, (dn, rn)
    lat.sort()
    stats = {"calls": len(lat), "p50_ms": round(lat[len(lat) // 2] * 1e3, 3), "p90_ms": round(lat[int(len(lat) * 0.9)] * 1e3, 3),
             "max_ms": round(lat[-1] * 1e3, 3), "doc": "synthetic CFN template, 8 resources", "rules": "cfg-2 pack files"}
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root:
        os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
        json.dump(stats, open(os.path.join(root, "gpurun_out", "ffi_latency.json"), "w"), indent=1)
    assert stats["p50_ms"] < 50, stats   # no per-call multi-hundred-MB allocations


def test_concurrent_callers_match_oracle():
    cases = _cases(32)
    errors = []

    def worker(k):
        try:
            for i in range(k, len(cases) * 2, 4):
                d, dn, r, rn, exp = cases[i % len(cases)]
                got = guard_amd.run_checks(d, dn, r, rn)
                if got != exp:
                    errors.append((k, dn, rn))
        except Exception as e:   # noqa: BLE001 -- reported through the assertion below
            errors.append((k, repr(e)))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]


def test_error_contract():
    # code / message / NULL result on error, like ffi-support's ExternError (guard-ffi/src/lib.rs:32-47)
    with pytest.raises(guard_amd.GuardError) as ei:
        guard_amd.run_checks("{", "bad.json", "Resources exists", "r.guard")
    # helper.rs:30-36: serde_json fails, then `serde_yaml::from_str(..)?` -> Error::YamlError, code 2;
    # the text after the Display prefix is libyaml's own problem string here, serde_yaml's there
    assert ei.value.code == 2
    assert ei.value.message.startswith("Error parsing incoming YAML context ")
