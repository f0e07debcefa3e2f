"""The native synthetic-corpus generator is byte-identical to synth.py (no GPU needed)."""
import guard_amd
import synth


def test_native_generator_matches_python():
    for i in list(range(40)) + [999, 123456, 999999]:
        assert guard_amd.synth_cfn_doc(i) == synth.cfn_corpus(1, start=i)[0], i


def test_native_generator_resource_counts():
    for nres in (0, 1, 7):
        assert guard_amd.synth_cfn_doc(5, nres) == synth.cfn_corpus(1, start=5, n_resources=nres)[0]


def test_native_yaml_generator_matches_python():
    """gg_synth_cfn_yaml_doc (synth_corpus.cpp) writes synth.cfn_yaml_doc's bytes, and the YAML reads back
    as the template cfn_doc builds"""
    import yaml
    for i in list(range(40)) + [12345, 999999]:
        assert guard_amd.synth_cfn_yaml_doc(i, 12) == synth.cfn_yaml_doc(i, 12), i
    for i in range(20):
        assert yaml.safe_load(synth.cfn_yaml_doc(i, 30)) == synth.cfn_doc(i, 30)


def test_synth_texts_inputs():
    """gg_synth_texts: the validate inputs the bench's streamed leg passes to cfn_guard_validate_batch_stream"""
    import ctypes
    for fmt, gen, ext in (("json", lambda i: synth.cfn_corpus(1, start=i, n_resources=6)[0], "json"),
                          ("yaml", lambda i: synth.cfn_yaml_doc(i, 6), "yaml")):
        t = guard_amd.SynthTexts(50, 12, n_resources=6, fmt=fmt, threads=3)
        try:
            for k in range(12):
                assert ctypes.string_at(t.inputs[k].content).decode() == gen(50 + k)
                assert ctypes.string_at(t.inputs[k].file_name).decode() == "synthetic-%d.%s" % (50 + k, ext)
        finally:
            t.close()
