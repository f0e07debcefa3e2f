"""The multi-device path's host logic, on the CPU: the byte-balanced document split and the join of
per-shard reports (cfn_guard_validate_batch_devices; SURVEY.md 8(b) n_gpus, 8(e)).

* gg_shard_by_bytes is the algorithm of sharding.shard_ranges_by_bytes (the torch.distributed path's
  split): the same ranges on random size vectors, min(n, shards) non-empty shards, the
  ranges contiguous and covering every document.
* gg_session_report_shards renders a session's results as shards and joins them exactly as the
  multi-device entry joins its devices' shards; on replayed MI355X results (tests/golden/replay, no GPU)
  the joined text and exit code must equal the one-piece report in all four formats, whatever the cuts
  (empty shards, one-document shards, ragged)."""
import os
import random
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "cloudformation-guard_amd"))
sys.path.insert(0, os.path.join(HERE, "golden"))
import guard_amd  # noqa: E402
import make_replay_fixtures as fx  # noqa: E402
import sharding  # noqa: E402


@pytest.mark.parametrize("seed", range(20))
def test_shard_split_matches_python_split(seed):
    r = random.Random(seed)
    n = r.choice([0, 1, 2, 3, 7, 64, 500])
    sizes = [r.choice([0, 1, 10, 1000, 100000]) if r.random() < 0.3 else r.randint(100, 20000) for _ in range(n)]
    for world in (1, 2, 3, 4, 8):
        got = guard_amd.shard_by_bytes(sizes, world)
        assert got == sharding.shard_ranges_by_bytes(sizes, world)
        assert sum(c for _, c in got) == n
        assert all(got[k][0] + got[k][1] == got[k + 1][0] for k in range(world - 1))
        assert sum(1 for _, c in got if c) == min(n, world)   # no shard idles while documents remain


def test_shard_split_balances_bytes():
    sizes = [random.Random(7).randint(1000, 9000) for _ in range(10000)]
    parts = guard_amd.shard_by_bytes(sizes, 8)
    per = [sum(sizes[f:f + c]) for f, c in parts]
    assert max(per) - min(per) <= 2 * max(sizes)


@pytest.mark.parametrize("name", sorted(fx.CASES))
@pytest.mark.parametrize("fmt", ["json", "yaml", "sarif", "junit"])
def test_joined_shard_reports_equal_one_report(name, fmt):
    s = fx.session(name)
    s.load_results(os.path.join(HERE, "golden", "replay", name + ".bin"))
    whole, code = s.report(fmt)
    n = s.stat(0)
    cuts_list = [[], [0], [n], [1], [n // 2], [n // 3, n // 3, 2 * n // 3], [1, 2, 3, n - 1], list(range(1, n))[:40]]
    for cuts in cuts_list:
        out, c = s.report_shards(fmt, cuts)
        assert c == code, cuts
        assert out == whole, (fmt, cuts)
    s.close()
