"""Host wall time against device time per call of the C2 steady-state tick (bench.py --config c2 --steady): for every
zb_step / zb_serialize of the timed ticks, the Python wall time, the engine's own wall time (zb_step_stats.wall_ms) and
the kernel time it measured. usage: python3 tools/gpu/steady_calls.py [ticks]"""
import functools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import bench  # noqa: E402
import bench_steady  # noqa: E402
from zeebe_amd import engine as zbe  # noqa: E402

ROWS = []
MEM = []


def main():
    ticks = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    step0, ser0 = zbe.Engine.step, zbe.Engine.serialize

    @functools.wraps(step0)
    def step(self, *a, **k):
        t = time.perf_counter()
        st = step0(self, *a, **k)
        ROWS.append(("step", (time.perf_counter() - t) * 1e3, st["wall_ms"], st["wave_kernel_ms"], st["launches"],
                     st["waves"]))
        m = self.memory_stats()
        MEM.append("arena_used %.0f MB of %.0f, rows %d, compactions %d" % (m["arena_used"] / 2**20,
                                                                          m["arena_bytes"] / 2**20,
                                                                          m["rows_allocated"], m["compactions"]))
        return st

    @functools.wraps(ser0)
    def serialize(self, *a, **k):
        t = time.perf_counter()
        s = ser0(self, *a, **k)
        ROWS.append(("serialize", (time.perf_counter() - t) * 1e3, s["wall_ms"],
                     s["write_kernel_ms"] + s["size_kernel_ms"], 0, 0))
        return s

    zbe.Engine.step, zbe.Engine.serialize = step, serialize
    sys.argv = sys.argv[:1]
    a = bench.parse()
    bench_steady.run_steady(a, 0, 1, 0, lambda: None, ticks, 1)
    print("%-10s %9s %9s %9s %8s %6s" % ("call", "py ms", "wall ms", "kernel ms", "launches", "waves"))
    for r in ROWS[-2 * ticks:]:
        print("%-10s %9.3f %9.3f %9.3f %8d %6d" % r)
    for m in MEM[-ticks - 2:]:
        print(m)


if __name__ == "__main__":
    main()
