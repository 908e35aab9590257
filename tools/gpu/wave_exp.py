"""Wave-pipeline stepping time of one bench workload under several zb_config flag sets, in one process on one box
(same-box A/B). usage: python3 tools/gpu/wave_exp.py [c2|c3|c4] [instances] [flags,flags,...]
Each flag set: 1 warm-up step + 3 timed steps of the general wave pipeline (no drain); prints stepping ms,
wave count and the summed wave-kernel time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import bench  # noqa: E402
from zeebe_amd.engine import Engine  # noqa: E402


def run(cfg, n, flags, a):
    xml, pid, blob, offs, jp, desc = bench.workload(cfg, n, 0, a.tasks)
    recs = bench.RECS_PER_INST[cfg](a.tasks)
    rows = {"c1": n * 3, "c2": n * (a.tasks + 2), "c3": n * 3, "c4": n * 20}[cfg]
    arena = {"c1": n * 96, "c2": n * (48 + 48 * a.tasks), "c3": n * 64, "c4": n * 1200}[cfg] + (64 << 20)
    eng = Engine(device=0, log_capacity=int(n * recs), row_capacity=int(rows), arena_bytes=int(arena), wave_only=True,
                 flags=flags)
    eng.deploy(xml, 100, 1)
    for act, p in jp.items():
        eng.set_job_payload(100, act, p)
    eng.create_packed(pid, blob, offs)
    out = []
    for it in range(4):
        eng.reset(keep_staged=True)
        t0 = time.perf_counter()
        st = eng.step()
        t1 = time.perf_counter()
        assert st["quiescent"], st
        if it:
            out.append(((t1 - t0) * 1e3, st["waves"], st["wave_kernel_ms"], st["transitions"]))
    eng.close()
    ms = sum(o[0] for o in out) / len(out)
    kms = sum(o[2] for o in out) / len(out)
    print("%s n=%d flags=%d: stepping %.2f ms (runs %s), waves %d, wave kernels %.2f ms, transitions %d" % (
        cfg, n, flags, ms, " ".join("%.2f" % o[0] for o in out), out[0][1], kms, out[0][3]), flush=True)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    fl = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
    sys.argv = sys.argv[:1]
    a = bench.parse()
    for f in fl:
        run(cfg, n, f, a)


if __name__ == "__main__":
    main()
