"""bench.py's full-size parity check (cpu_baseline): each core's structured JSON report is joined from the
oracle's one-document reports (the serde pretty layout) and compared, by digest, with the GPU session's
report of the same document range.  The join must equal the oracle's report of the whole range."""
import hashlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cloudformation-guard_amd")]

import bench  # noqa: E402
import rulepack  # noqa: E402
from guard_oracle import validate_structured  # noqa: E402


@pytest.mark.parametrize("workload,first,n", [("cfg2", 7, 3), ("cfg5", 11, 4)])
def test_joined_sample_report_equals_the_range_report(workload, first, n):
    _, _, evals, f0, statuses, report = bench._oracle_worker((workload, first, n, 20))
    rules = rulepack.rule_pack(workload)
    prefix = {"cfg4": "plan", "cfg5": "snapshot"}.get(workload, "synthetic")
    docs = bench._workload_docs(workload, first, n, 20)
    text, code, _ = validate_structured(rules, [("%s-%d.json" % (prefix, first + i), d) for i, d in enumerate(docs)])
    assert (f0, evals, len(statuses)) == (first, n * len(rules), n * len(rules))
    assert report == (first, n, hashlib.sha256(text.encode()).hexdigest(), len(text), code)
