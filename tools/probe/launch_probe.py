"""Per-operation cost (us, back to back on one stream, one synchronisation at the end) of the HIP runtime this
process binds: `python3 tools/probe/launch_probe.py sys` binds the system ROCm runtime (as bench.py does),
`... torch` torch's bundled copy (import torch first). Measurement tool; build: make -C tools/probe."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if sys.argv[1:] == ["torch"]:
    import torch  # noqa: F401
L = ctypes.CDLL(os.path.join(HERE, "liblaunchprobe.so"))
L.probe.restype = ctypes.c_double
L.probe_runtime.restype = ctypes.c_char_p
print("runtime:", L.probe_runtime().decode())
names = ["empty kernel", "kernel, 768 B args", "memset 64 B", "D2H copy 64 B", "kernel + sync", "kernel 4096 WGs",
         "event record", "kernel, 2 KB args"]
for k, name in enumerate(names):
    L.probe(k, 200)
    v = min(L.probe(k, 2000 if k != 4 else 500) for _ in range(3))
    print("%-22s %8.2f us" % (name, v))
