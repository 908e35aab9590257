"""Summarise the rocprofv3 PMC passes of run_gpu_pmc.sh (one counter set per pass directory p<i>).

Per kernel (averaged over its dispatches) every counter of every pass, plus derived figures:
  hbm_bytes        2 * FETCH_SIZE + WRITE_SIZE (both reported in KB; gfx950 tallies 128-B read requests
                   at 64 B, so FETCH_SIZE is doubled -- MI355X_MICROARCH.md, HBM / rocprofv3 section)
  kernel_cycles    GRBM_GUI_ACTIVE / 8 (the counter is summed over the 8 XCDs)
  valu_busy        SQ_ACTIVE_INST_VALU * 4 / (#SIMD = 4 * 256 CUs) / kernel_cycles (gfx94x formula)
  valu_lane_util   SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU): mean active lanes of a VALU
                   instruction (1.0 = no divergence)
  mean_waves_cu    4 * SQ_WAVE_CYCLES / kernel_cycles / 256 CUs: resident waves per CU averaged over the
                   kernel (SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, MI355X_MICROARCH.md;
                   of 32; occupancy = mean_waves_cu / 32). SQ_ACCUM_PREV_HIRES reads 0 on gfx950 / ROCm 7.2.
  wait_frac        SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  lds_conflict     SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE

usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> profiles/r02/pmc_<tag>.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CUS = 256
XCDS = 8


def per_kernel(pass_dir):
    """PMC_SKIP_TICKS=k (environment): drop every dispatch before the (k+1)-th k_inject, i.e. the run's first k ticks
    (the steady-state bench's population tick)."""
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(set))
    rows = []
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    skip = int(os.environ.get("PMC_SKIP_TICKS", "0"))
    if skip:
        did = lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)  # noqa: E731
        inj = sorted({did(r) for r in rows if "k_inject" in r["Kernel_Name"]})
        first = inj[skip] if len(inj) > skip else float("inf")
        rows = [r for r in rows if did(r) >= first]
    if True:
        if True:
            for row in rows:
                k = row["Kernel_Name"]
                c = row.get("Counter_Name")
                acc[k][c] += float(row["Counter_Value"])
                calls[k][c].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return {k: {c: acc[k][c] / max(len(calls[k][c]), 1) for c in acc[k]} for k in acc}, \
        {k: max(len(v) for v in calls[k].values()) for k in calls}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kernels = defaultdict(dict)
    dispatches = {}
    sets = []
    for d in sorted(glob.glob(os.path.join(src, "p*")), key=lambda p: int(''.join(ch for ch in os.path.basename(p) if ch.isdigit()) or 0)):
        if not os.path.isdir(d):
            continue
        setf = d + ".set"
        if os.path.exists(setf):
            sets.append(open(setf).read().strip())
        vals, n = per_kernel(d)
        for k, cs in vals.items():
            kernels[k].update(cs)
            dispatches[k] = max(dispatches.get(k, 0), n[k])
    out = {}
    for k, c in kernels.items():
        if "zbg::" not in k:
            continue
        d = dict(c)
        d["dispatches"] = dispatches.get(k, 0)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes"] = 1024 * (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"])
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs: one XCD's value is the kernel's duration in cycles
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / XCDS
        if cyc:
            d["kernel_cycles"] = cyc
        if cyc and "SQ_ACTIVE_INST_VALU" in c:
            d["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (4 * CUS) / cyc
        if cyc and "SQ_WAVE_CYCLES" in c:
            d["mean_waves_cu"] = 4 * c["SQ_WAVE_CYCLES"] / cyc / CUS  # quad-cycles
            d["occupancy"] = d["mean_waves_cu"] / 32.0
        if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
            d["valu_lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
        if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in c:
            d["wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
            d["lds_conflict"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
        out[k] = d
    res = {"source": src, "passes": sets, "occupancy_units": "quad-cycle corrected",
           "correction": "FETCH_SIZE doubled (gfx950 tallies 128-B requests at 64 B); WRITE_SIZE as reported",
           "kernels": out}
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    for k, d in sorted(out.items(), key=lambda kv: -kv[1].get("hbm_bytes", 0)):
        print(k[:60], {x: round(d[x], 4) for x in ("hbm_bytes", "valu_busy", "valu_lane_util", "occupancy",
                                                     "wait_frac", "lds_conflict", "kernel_cycles", "dispatches") if x in d})


def rederive(path):
    """Recompute mean_waves_cu / occupancy of a summary written before the quad-cycle correction."""
    with open(path) as f:
        res = json.load(f)
    if res.get("occupancy_units") == "quad-cycle corrected":
        return
    for d in res["kernels"].values():
        if d.get("kernel_cycles") and "SQ_WAVE_CYCLES" in d:
            d["mean_waves_cu"] = 4 * d["SQ_WAVE_CYCLES"] / d["kernel_cycles"] / CUS
            d["occupancy"] = d["mean_waves_cu"] / 32.0
    res["occupancy_units"] = "quad-cycle corrected"
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--rederive":
        for p in sys.argv[2:]:
            rederive(p)
    else:
        main()
