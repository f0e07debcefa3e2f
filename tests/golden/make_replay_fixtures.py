"""Device-output fixtures for the CPU report-writer parity test (tests/test_report_replay_cpu.py).

Run on a GPU box (python tests/golden/make_replay_fixtures.py): evaluates each pack below over its
documents on the MI355X and saves the raw device results (tile headers, rule statuses, failure records)
with Session.save_results.  The CPU test reloads them into a session with the same rules and documents
and renders every report format on the host.  The records reference compiled clause ids: regenerate
after a change to the rules compiler."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import synth  # noqa: E402

CASES = {
    # name: (rule pack dir, documents, document name prefix)
    "cfg3": ("cfg3_rulepack", lambda: synth.cfn_corpus(24, start=4242, n_resources=50), "t"),
    "capture": ("capture_rulepack", lambda: synth.cfn_corpus(16, start=77, n_resources=12), "c"),
}


def pack(d):
    p = os.path.join(HERE, d)
    return [(f, open(os.path.join(p, f)).read()) for f in sorted(os.listdir(p)) if f.endswith(".guard")]


def session(name):
    d, docs, prefix = CASES[name]
    s = guard_amd.Session()
    for f, text in pack(d):
        s.add_rules(text, f)
    docs = docs()
    s.add_docs(docs, ["%s-%d.json" % (prefix, i) for i in range(len(docs))])
    return s


if __name__ == "__main__":
    for name in CASES:
        s = session(name)
        s.eval(1)
        out = os.path.join(HERE, "replay", name + ".bin")
        s.save_results(out)
        s.close()
        print("saved", out, os.path.getsize(out))
