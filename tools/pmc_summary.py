"""Summarise the rocprofv3 PMC passes of run_gpu_pmc.sh into profiles/<round>/pmc_<tag>.json.

Pass 1 collects FETCH_SIZE, pass 2 WRITE_SIZE (separate runs, kernel trace only). Both are reported
in KB per dispatch; gfx950 tallies 128-B read requests at 64 B, so FETCH_SIZE is doubled
(MI355X_MICROARCH.md, HBM/rocprofv3 section). WRITE_SIZE is taken as reported.

usage: python tools/pmc_summary.py gpurun_out/pmc profiles/r01/pmc_v5.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

MAIN_PREFERENCE = ("zbg::k_tmpl<false, false>", "zbg::k_tmpl<true, false>")


def per_kernel(pass_dir, counter):
    acc, calls = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = row["Kernel_Name"]
                acc[k] += float(row["Counter_Value"])
                calls[k].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return {k: acc[k] / max(len(calls[k]), 1) for k in acc}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    fetch = per_kernel(os.path.join(src, "p1"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "p2"), "WRITE_SIZE")
    kernels = {k: {"FETCH_SIZE_KB": fetch.get(k, 0.0), "WRITE_SIZE_KB": write.get(k, 0.0)}
               for k in sorted(set(fetch) | set(write)) if k.startswith(("zbg::", "void zbg::"))}
    main_k = None
    for pref in MAIN_PREFERENCE:
        main_k = next((k for k in kernels if pref in k), None)
        if main_k:
            break
    if main_k is None:
        main_k = max(kernels, key=lambda k: kernels[k]["WRITE_SIZE_KB"])
    fb = 2 * 1024 * kernels[main_k]["FETCH_SIZE_KB"]
    wb = 1024 * kernels[main_k]["WRITE_SIZE_KB"]
    out = {"command": "rocprofv3 --pmc <FETCH_SIZE | WRITE_SIZE> --kernel-trace -- python3 bench.py --steps 1 "
                      "--warmup 0 --instances 1000000 --no-cpu-baseline (one pass per counter, run_gpu_pmc.sh)",
           "workload": "C2: 20-task chain, 1,000,000 instances, one step",
           "kernels": kernels,
           "correction": "FETCH_SIZE doubled (gfx950 tallies 128-B requests at 64 B); WRITE_SIZE as reported",
           "main_kernel": main_k, "main_traffic_bytes": fb + wb,
           "main_fetch_bytes_corrected": fb, "main_write_bytes": wb}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("main_kernel", "main_traffic_bytes", "main_fetch_bytes_corrected",
                                          "main_write_bytes")}))


if __name__ == "__main__":
    main()
