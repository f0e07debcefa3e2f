"""The evaluator over an explicit continuation stack (csrc/eval_machine.inc, build variant "machine",
GG_MACHINE=1): no recursion, a static kernel stack.  Its library is loaded in a child process (GG_LIB) and
every report is compared with the CPU oracle over the cfg2-cfg5 packs and the edge / capture / count /
converter / NFA / word-boundary packs -- the same evaluation as the default recursive evaluator
(eval_recursive.inc), which the rest of the GPU suite runs."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cloudformation-guard_amd", "libcfnguard_mi355x_machine.so")


def test_machine_build_matches_oracle():
    if not os.path.exists(LIB):
        pytest.fail("machine build missing: python cloudformation-guard_amd/build.py machine")
    env = dict(os.environ, GG_LIB=LIB)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "machine_gpu_child.py")], env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count("ok ") >= 5
