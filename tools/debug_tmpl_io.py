"""Debug aid: C3 with n instances through the instance-order and the class-uniform emit; prints the first
descriptor / record differences."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from zeebe_amd import workloads  # noqa: E402


def run(io, n):
    from zeebe_amd.engine import CFG_INSTANCE_ORDER, CFG_NO_DEFER, Engine
    cfg = workloads.CONFIGS["c3"]
    blob, offs = cfg["payloads"](n)
    e = Engine(flags=CFG_NO_DEFER | (CFG_INSTANCE_ORDER if io else 0))
    e.deploy(cfg["workflow"]().to_xml(), 100, 1)
    e.create(cfg["process"], workloads.split(blob, offs))
    st = e.step()
    d = e.descriptors()
    recs = e.records()
    e.close()
    return st, d, recs


if len(sys.argv) > 2:  # survey: bad descriptor counts for several sizes
    for n in map(int, sys.argv[1:]):
        _, a, _ = run(1, n)
        _, b, _ = run(0, n)
        bad = [i for i in range(len(b)) if a[i].tobytes() != b[i].tobytes()]
        print("n", n, "bad", len(bad), "first", bad[:3], "payload io/cls", [(int(a[i]["payload"]), int(b[i]["payload"])) for i in bad[:2]])
    sys.exit(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
s1, d1, r1 = run(1, n)
s0, d0, r0 = run(0, n)
print("stats io", {k: s1[k] for k in ("transitions", "records_written", "path")}, "cls", {k: s0[k] for k in ("transitions", "records_written", "path")})
bad = 0
for i in range(min(len(d0), len(d1))):
    if d0[i].tobytes() != d1[i].tobytes() or r0[i] != r1[i]:
        print(i, "cls", d0[i], r0[i].value[:60], "\n   io ", d1[i], r1[i].value[:60], r1[i].source_position)
        bad += 1
        if bad > 6:
            break
print("len", len(d0), len(d1), "bad", bad)
print("CREATE payload refs io", [int(x) for x in d1["payload"][:3]], "cls", [int(x) for x in d0["payload"][:3]])
print("first emitted io", d1[n:n + 4], "\ncls", d0[n:n + 4])
