"""Host report writers against the oracle, on saved device results (no GPU needed).

tests/golden/replay/*.bin hold the raw results of MI355X evaluations (tile headers, rule statuses,
failure records; tests/golden/make_replay_fixtures.py).  Each is reloaded into a session with the same
rules files and documents, and the host renders every `validate --structured` format from it; the text
must equal the oracle's for the same inputs (reporters/validate/structured.rs, sarif.rs, xml.rs via
oracle/guard_oracle).  This pins the product's report writers (csrc/reporter.cpp) on the CPU suite,
including the streamed JSON writer and side records (join reasons R4 / R5 in the capture pack)."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_replay_fixtures as fx  # noqa: E402
from guard_oracle import validate_structured as oracle_validate  # noqa: E402


@pytest.mark.parametrize("name", sorted(fx.CASES))
@pytest.mark.parametrize("fmt", ["json", "yaml", "sarif", "junit"])
def test_replayed_device_results_report_like_oracle(name, fmt):
    d, docs, prefix = fx.CASES[name]
    docs = docs()
    data = [("%s-%d.json" % (prefix, i), t) for i, t in enumerate(docs)]
    exp, ecode, _ = oracle_validate(fx.pack(d), data, output=fmt)
    s = fx.session(name)
    s.load_results(os.path.join(HERE, "golden", "replay", name + ".bin"))
    out, code = s.report(fmt)
    s.close()
    assert code == ecode
    assert out == exp
