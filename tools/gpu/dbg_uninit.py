"""Debug aid: run a scenario with the product library and with the guard-band build (every allocation filled with
0xA5), in two child processes, and print the first records whose descriptors / value lengths / values differ --
a difference means a kernel read device memory nothing wrote."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SCEN = sys.argv[1] if len(sys.argv) > 1 else "size"


def scenario():
    import msgpack
    from zeebe_amd import bpmn, workloads
    from zeebe_amd.engine import CFG_GENERIC_DRAIN, Engine

    if SCEN == "size":
        wf = bpmn.chain_workflow(4)
        blob, offs = workloads.order_payloads(300)
        jp = {"t%d" % k: msgpack.packb({"k%d" % k: "y" * (7 * k)}) for k in range(1, 5)}
        e = Engine(wave_only=True, log_capacity=1 << 16, row_capacity=1 << 12, arena_bytes=16 << 20)
    else:
        wf = bpmn.chain_workflow(6)
        blob, offs = workloads.order_payloads(400)
        jp = {"t%d" % k: msgpack.packb({"k%d" % k: "x" * (40 * k * k // 3)}) for k in range(1, 7)}
        e = Engine(flags=0 if SCEN == "fast" else CFG_GENERIC_DRAIN, log_capacity=1 << 16, row_capacity=1 << 12,
                   arena_bytes=16 << 20)
    e.deploy(wf.to_xml(), 100, 1)
    for act, p in jp.items():
        e.set_job_payload(100, act, p)
    e.create_packed("chain", blob, offs)
    e.step()
    n = e.log_size()
    d = e.descriptors(0, n)
    recs = e.records(0, n)
    out = []
    for i in range(n):
        r = recs[i]
        out.append([int(d["key"][i]), int(d["scope_key"][i]), int(d["inst_key"][i]), int(d["payload"][i]),
                    int(d["elem"][i]), int(d["intent"][i]), int(d["kind"][i]), r.source_position, len(r.value),
                    r.value.hex()])
    print(json.dumps(out))


if __name__ == "__main__":
    if os.environ.get("DBG_CHILD"):
        scenario()
        sys.exit(0)
    res = {}
    for checked in ("0", "1"):
        env = dict(os.environ, DBG_CHILD="1", ZB_CHECKED_LIBRARY=checked)
        p = subprocess.run([sys.executable, __file__, SCEN], env=env, capture_output=True, text=True, timeout=200)
        if p.returncode != 0:
            print("child failed", checked, p.stderr[-3000:])
            sys.exit(1)
        res[checked] = json.loads(p.stdout.strip().splitlines()[-1])
    a, b = res["0"], res["1"]
    print("records", len(a), len(b))
    shown = 0
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            print("pos", i, "product:", x[:9], x[9][:160])
            print("        checked:", y[:9], y[9][:160])
            src = x[7]
            if src >= 0:
                print("   source", src, a[src][:9])
            shown += 1
            if shown >= 6:
                break
    print("differences:", sum(1 for x, y in zip(a, b) if x != y))
