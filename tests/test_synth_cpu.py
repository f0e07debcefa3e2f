"""The native synthetic-corpus generator is byte-identical to synth.py (no GPU needed)."""
import guard_amd
import synth


def test_native_generator_matches_python():
    for i in list(range(40)) + [999, 123456, 999999]:
        assert guard_amd.synth_cfn_doc(i) == synth.cfn_corpus(1, start=i)[0], i


def test_native_generator_resource_counts():
    for nres in (0, 1, 7):
        assert guard_amd.synth_cfn_doc(5, nres) == synth.cfn_corpus(1, start=5, n_resources=nres)[0]
