"""Per-dispatch HBM traffic of the evaluation kernel from rocprofv3 --pmc passes.

FETCH_SIZE / WRITE_SIZE are in KiB.  Correction per MI355X_MICROARCH.md "HBM": on gfx950
FETCH_SIZE reports half the bytes of a 16 B/lane coalesced read, so it is doubled; WRITE_SIZE is
taken as is.  Other access widths are uncalibrated (the guide says so), so the raw counters are
kept next to the corrected figure.  Usage: python tools/pmc_summary.py gpurun_out/pmc
"""
import collections
import csv
import glob
import json
import os
import sys

KERNEL = "guard_eval_lanes_kernel"


def main(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            name = "lanes" if KERNEL in k else ("resource_type" if "resource_type_kernel" in k else
                                                ("rule_count" if "rule_count_kernel" in k else None))
            if name:
                per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for name, ctrs in per.items():
        row = {c: sum(v) / len(v) for c, v in ctrs.items()}
        out[name] = {"fetch_kib_raw": row.get("FETCH_SIZE"), "write_kib_raw": row.get("WRITE_SIZE"),
                     "dispatches": max(len(v) for v in ctrs.values()),
                     "counters_mean_per_dispatch": {c: v for c, v in sorted(row.items())
                                                    if c not in ("FETCH_SIZE", "WRITE_SIZE")}}
    lanes = out.get("lanes", {})
    hbm = None
    if lanes.get("fetch_kib_raw") is not None and lanes.get("write_kib_raw") is not None:
        hbm = int(2 * lanes["fetch_kib_raw"] * 1024 + lanes["write_kib_raw"] * 1024)
    # the workload string bench.py printed in the profiled run (its config.workload), so bench.py's
    # load_pmc finds this summary for exactly that workload
    wl = os.environ.get("PMC_WORKLOAD")
    for log in sorted(glob.glob(os.path.join(d, "*.log"))):
        for line in open(log, errors="replace"):
            if line.startswith('{"metric"') and not wl:
                try:
                    wl = json.loads(line)["config"]["workload"]
                except Exception:
                    pass
    res = {"workload": wl or "cfg2: 1000000 synthetic CFN templates/GPU (50 resources) x 7-file rule pack",
           "kernel": "gg::guard_eval_lanes_kernel",
           "hbm_bytes_per_launch": hbm,
           "correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM section",
           "kernels": out}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
