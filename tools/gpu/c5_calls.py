"""Host wall time per engine call of the C5 bench step (bench.py --config c5), to find the time the kernel trace
does not show (host work between kernels). usage: python3 tools/gpu/c5_calls.py [instances] [steps]"""
import collections
import functools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if os.environ.get("ZB_SYSRT"):  # bind the system HIP runtime first, as bench.py's main does
    from zeebe_amd.engine import lib  # noqa: E402

    lib()

import bench  # noqa: E402
from zeebe_amd import engine as zbe  # noqa: E402

T = collections.defaultdict(lambda: [0, 0.0])
SEQ = []
TIMED = ("step", "comm_pending", "comm_exchange", "publish_uploaded", "serialize", "reset", "create",
         "upload_staged", "upload_publishes_packed")


def _wrap(name, f):
    @functools.wraps(f)
    def g(*args, **kw):
        t = time.perf_counter()
        try:
            return f(*args, **kw)
        finally:
            T[name][0] += 1
            T[name][1] += time.perf_counter() - t
            SEQ.append((name, t, time.perf_counter() - t))
    return g


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for name in TIMED:
        setattr(zbe.Engine, name, _wrap(name, getattr(zbe.Engine, name)))
    sys.argv = sys.argv[:1] + ["--config", "c5", "--instances", str(n), "--steps", str(steps), "--warmup", "1",
                               "--no-cpu-baseline"]
    a = bench.parse()
    bench.run_c5(a, 0, 1, 0, None)
    resets = [i for i, x in enumerate(SEQ) if x[0] == "reset"] + [len(SEQ)]
    spans = []
    for a_, b_ in zip(resets, resets[1:]):  # the timed part: first step call .. the serialize's end
        seg = SEQ[a_:b_]
        s0 = next(t for name, t, d in seg if name == "step")
        s1 = max(t + d for name, t, d in seg if name == "serialize")
        spans.append((s1 - s0) * 1e3)
    print("timed span per step (ms):", " ".join("%.3f" % x for x in spans))
    last = resets[-2]
    t0 = SEQ[last][1]
    print("last step, call by call (start ms, duration ms):")
    for name, t, d in SEQ[last:]:
        print("  %8.3f %8.3f %s" % ((t - t0) * 1e3, d * 1e3, name))
    print("per call (all steps incl. warmup, %d steps):" % (steps + 1))
    for k, (c, s) in sorted(T.items(), key=lambda x: -x[1][1]):
        print("  %-26s %5d calls %9.2f ms total %8.3f ms/call" % (k, c, s * 1e3, s * 1e3 / max(c, 1)))


if __name__ == "__main__":
    main()
