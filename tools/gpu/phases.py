"""k_wave's time per phase (process + tile scan / look-back / emit) on a bench workload, from the ZB_PHASES
measurement build (zeebe_amd/csrc Makefile target `phases`). usage: ZB_PHASES_LIBRARY=1 python3 tools/gpu/phases.py
[c2|c3|c4] [instances]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["ZB_PHASES_LIBRARY"] = "1"

import bench  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    sys.argv = sys.argv[:1]
    a = bench.parse()
    a.wave_only = True
    a.config = cfg
    xml, pid, blob, offs, jp, desc = bench.workload(cfg, n, 0, a.tasks)
    eng = bench.make_engine(cfg, n, a, 0, 1, 0)
    eng.deploy(xml, 100, 1)
    for act, p in jp.items():
        eng.set_job_payload(100, act, p)
    eng.create_packed(pid, blob, offs)
    for it in range(3):
        eng.reset(keep_staged=True)
        p0 = eng.phase_times()
        t0 = time.perf_counter()
        st = eng.step()
        t1 = time.perf_counter()
        p1 = eng.phase_times()
        d = {k: p1[k] - p0[k] for k in p1}
        tot = d["process"] + d["lookback"] + d["emit"]
        print("step %d: %.2f ms, waves %d, wave kernels %.2f ms; tiles %d; per tile us: process %.2f lookback %.2f "
              "emit %.2f; shares %.2f / %.2f / %.2f; look-back rounds per tile %.1f" % (
                  it, (t1 - t0) * 1e3, st["waves"], st["wave_kernel_ms"], d["tiles"],
                  d["process"] / 100 / max(d["tiles"], 1), d["lookback"] / 100 / max(d["tiles"], 1),
                  d["emit"] / 100 / max(d["tiles"], 1), d["process"] / tot, d["lookback"] / tot, d["emit"] / tot,
                  d["rounds"] / max(d["tiles"], 1)),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
