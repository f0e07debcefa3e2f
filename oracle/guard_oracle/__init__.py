"""guard_oracle -- CPU restatement of cfn-guard's (document x rules-file) evaluation path.

TEST INFRASTRUCTURE ONLY.  This package is the parity oracle for the MI355X build.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker.  The product path (``cloudformation-guard_amd/``) never imports,
links or executes anything under ``oracle/``.

Reference: joshfried-aws/cloudformation-guard v3.1.2 (guard/src/rules/*).  Pinned against the
reference's own golden files (guard/resources/validate/output-dir/structured.json, ...) and
test expectations (guard-examples/**/*-tests.yaml); see tests/test_oracle_*.py.
"""
from .errors import GuardError  # noqa: F401
from .report import validate_structured, run_checks  # noqa: F401
