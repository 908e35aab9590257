"""k_tdrain_write's time per phase (generation setup / headers / encode / image stream) on the C3 headline step, from
the ZB_PHASES measurement build (zeebe_amd/csrc Makefile target `phases`).
usage: python3 tools/gpu/tdrain_phases.py [instances]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["ZB_PHASES_LIBRARY"] = "1"

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    sys.argv = sys.argv[:1]
    a = bench.parse()
    xml, pid, blob, offs, jp, desc = bench.workload("c3", n, 0, a.tasks)
    eng = bench.make_engine("c3", n, a, 0, 1, 0)
    eng.deploy(xml, 100, 1)
    for act, p in jp.items():
        eng.set_job_payload(100, act, p)
    eng.create_packed(pid, blob, offs)
    del blob
    for it in range(3):
        eng.reset(keep_staged=True)
        st = eng.step()
        p0 = eng.tdrain_phase_times()
        t0 = time.perf_counter()
        ser = eng.serialize(n, eng.log_size() - n)
        t1 = time.perf_counter()
        p1 = eng.tdrain_phase_times()
        d = {k: p1[k] - p0[k] for k in p1}
        tot = d["setup"] + d["headers"] + d["encode"] + d["stream"]
        w = max(d["waves"], 1)
        print("drain %d: %.2f ms (write kernel %.2f ms), waves %d, generations per wave %.1f; per wave us: setup %.2f "
              "headers %.2f encode %.2f stream %.2f; shares %.2f / %.2f / %.2f / %.2f" % (
                  it, (t1 - t0) * 1e3, ser["write_kernel_ms"], d["waves"], d["gens"] / w,
                  d["setup"] / 100 / w, d["headers"] / 100 / w, d["encode"] / 100 / w, d["stream"] / 100 / w,
                  d["setup"] / tot, d["headers"] / tot, d["encode"] / tot, d["stream"] / tot), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
