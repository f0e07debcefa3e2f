"""One streamed C-ABI leg of bench.py in a process of its own (the way a caller process uses the entry):
cfn_guard_validate_batch_stream (devices = 0) or cfn_guard_validate_batch_stream_devices over devices
0..devices-1, on `docs` synthetic templates of the bench workload, the report counted by the library's native
callback; an optional 9th argument names the output format (json, yaml, sarif, junit: the other formats go
through cfn_guard_validate_batch_stream_ex).  Prints one JSON line: seconds, report_bytes, exit_code, gen_s."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cloudformation-guard_amd"), os.path.join(ROOT, "tests")]
import guard_amd  # noqa: E402
import rulepack  # noqa: E402


def main():
    workload, first, docs, resources, fmt, chunk, devices, threads = sys.argv[1:9]
    first, docs, resources, chunk, devices, threads = int(first), int(docs), int(resources), int(chunk), int(devices), int(threads)
    output = sys.argv[9] if len(sys.argv) > 9 else "json"
    rules = rulepack.rule_pack(workload)
    t0 = time.time()
    texts = guard_amd.SynthTexts(first, docs, n_resources=resources, fmt=fmt, threads=threads)
    gen_s = time.time() - t0
    nb = [0]

    def count(n):
        nb[0] += n
    try:
        t0 = time.time()
        _, code = guard_amd.validate_structured_stream(rules, None, write=count, chunk_docs=chunk, inputs=texts.inputs,
                                                       n_docs=texts.n, count_only="native",
                                                       devices=(list(range(devices)) if devices else False), output=output)
        dt = time.time() - t0
    finally:
        texts.close()
    print(json.dumps({"seconds": dt, "report_bytes": nb[0], "exit_code": code, "gen_s": gen_s}), flush=True)


if __name__ == "__main__":
    main()
