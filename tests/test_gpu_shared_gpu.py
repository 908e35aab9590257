"""ZB_CFG_SHARED_GPU: the wave pipeline's persistent kernel (k_wave, zb_wave.hip) claims its tiles from a counter instead
of dealing them round-robin, so its hand-off progresses when other processes hold part of the GPU
(DESIGN.md section 6). The claimed order must give the same log, byte for byte:
  * against the round-robin deal, on a wave of more than two rounds of tiles (600k CREATE commands: 2344 tiles over
    a grid of at most 2048 workgroups) -- values and record headers of the whole drain;
  * against the oracle engine, record for record, on the fork / join workflow with scopes (C4's shape);
  * four processes stepping C4 on the one GPU at once (what the flag is for), every process the same log.
The eight-process bench run on one GPU: profiles/r06/c4_8rank_samedevice_r06final3.json.
"""
import numpy as np
import pytest

import test_gpu_parity
from test_gpu_parity import _compare, _run_both
from zeebe_amd import bpmn, workloads

pytestmark = pytest.mark.gpu


def _drain_all(flags, n):
    from zeebe_amd.engine import HEADER_DTYPE, Engine

    wf = bpmn.Bpmn.create_executable_process("p").start_event("s").end_event("e").done()
    e = Engine(wave_only=True, flags=flags, log_capacity=n * 10, row_capacity=n * 3, arena_bytes=n * 256 + (64 << 20))
    e.deploy(wf.to_xml(), 100, 1)
    blob, offs = workloads.order_payloads(n)
    e.create_packed("p", blob, offs)
    st = e.step()
    assert st["quiescent"] and st["completed_instances"] == n, st
    count = e.log_size()
    ser = e.serialize(0, count)
    vals = np.empty(max(ser["value_bytes"], 1), dtype=np.uint8)
    hdrs = np.empty(count, dtype=HEADER_DTYPE)
    e.drain_copy(vals.ctypes.data, 0, ser["value_bytes"], hdrs.ctypes.data)
    e.close()
    return st, hdrs, vals


def test_tile_claims_match_round_robin_deal():
    from zeebe_amd.engine import CFG_SHARED_GPU

    n = 600_000
    st_a, h_a, v_a = _drain_all(0, n)
    st_b, h_b, v_b = _drain_all(CFG_SHARED_GPU, n)
    assert st_a["transitions"] == st_b["transitions"] and st_a["waves"] == st_b["waves"]
    assert len(h_a) == len(h_b) and np.array_equal(h_a.view(np.uint8), h_b.view(np.uint8))
    assert len(v_a) == len(v_b) and np.array_equal(v_a, v_b)


def test_tile_claims_fork_join_vs_oracle(monkeypatch):
    from zeebe_amd.engine import CFG_SHARED_GPU

    monkeypatch.setitem(test_gpu_parity._CASE, "flags", CFG_SHARED_GPU)
    blob, offs = workloads.order_payloads(1500)
    payloads = [blob[offs[i]:offs[i + 1]] for i in range(1500)]
    o, e, _ = _run_both(bpmn.parallel_workflow(8).to_xml(), "par", payloads, path="wave",
                        log_capacity=1 << 20, row_capacity=1 << 16, arena_bytes=256 << 20)
    _compare(o, e)
    e.close()


_CHILD = r"""
import hashlib, os, sys, time
import numpy as np
sys.path[:0] = [os.environ["ZB_ROOT"]]
from zeebe_amd import bpmn, workloads
from zeebe_amd.engine import CFG_SHARED_GPU, HEADER_DTYPE, Engine
n, steps, me, peers, gate = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
e = Engine(wave_only=True, flags=CFG_SHARED_GPU, log_capacity=n * 200, row_capacity=n * 20,
           arena_bytes=n * 1200 + (64 << 20))
e.deploy(bpmn.parallel_workflow(8).to_xml(), 100, 1)
blob, offs = workloads.order_payloads(n)
e.create_packed("par", blob, offs)
open(os.path.join(gate, me), "w").close()
t0 = time.time()
while len(os.listdir(gate)) < peers:  # (all processes step at the same time)
    assert time.time() - t0 < 120, "peers did not start"
    time.sleep(0.01)
digests = set()
for _ in range(steps):
    e.reset(keep_staged=True)
    st = e.step()
    assert st["quiescent"] and st["completed_instances"] == n, st
    count = e.log_size()
    h = hashlib.sha256(b"%d %d" % (count, st["transitions"]))
    for start in (0, count // 2, count - (1 << 16)):  # (three 64k-record windows of the ~25M-record log)
        ser = e.serialize(start, 1 << 16)
        vals = np.empty(max(ser["value_bytes"], 1), dtype=np.uint8)
        hdrs = np.empty(1 << 16, dtype=HEADER_DTYPE)
        e.drain_copy(vals.ctypes.data, 0, ser["value_bytes"], hdrs.ctypes.data)
        h.update(hdrs.tobytes() + vals.tobytes())
    digests.add(h.hexdigest())
e.close()
assert len(digests) == 1, digests
print("digest", digests.pop())
"""


def test_processes_sharing_one_gpu(tmp_path):
    """Four processes step wave-only C4 batches (125k instances: waves of up to ~1M records, more than two rounds of
    tiles) on the one GPU at the same time, each k_wave grid sized for the whole device, so only part of each is
    resident: every step completes, and every process writes the same log every step (record
    count, transitions and three 64k-record windows of values and headers, byte for byte)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gate = tmp_path / "gate"
    gate.mkdir()
    env = dict(os.environ, ZB_ROOT=root)
    procs = [subprocess.Popen([sys.executable, "-c", _CHILD, "125000", "4", "p%d" % k, "4", str(gate)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for k in range(4)]
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=240)
            assert p.returncode == 0, (p.returncode, out[-2000:], err[-4000:])
            outs.append(out.split()[-1])
    finally:
        for p in procs:  # (a failed or timed-out case leaves no process on the GPU)
            if p.poll() is None:
                p.kill()
                p.wait()
    assert len(set(outs)) == 1, outs
