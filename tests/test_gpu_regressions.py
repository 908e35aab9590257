"""Regressions of device faults, each driven through the exact buffer sequence that produced it.

Uninitialised CREATE rows (round-3 fault in test_many_ticks_through_small_capacities): a CREATE
command allocates its instance's row in the wave that processes it, but the instance enters the index only when its
CREATED event is processed, one wave later. k_children (the first-live-child lookup of a cancellation, zb_wave.hip)
scans every allocated row, so when a CANCEL's TERMINATING is in the same wave as new CREATED events it read rows whose
memory still held whatever was there before -- a compacted-away row, another engine's data -- and indexed raux[] with
that garbage parent. The fault came and went with the allocator's layout. The guard-band build fills every fresh
allocation with 0xA5, which turns such a read into a certain fault (parent 0xa5a5a5a5), so the case runs there, in a
child process, as well as on the product build.

A log overflow in the middle of a tick (round-6 fault, found by test_gpu_shared_gpu.py with too small a log): the
wave that runs past the log window stops emitting at its end and flags DE_LOG_FULL, but its header still carries the
unbounded end / generation end, and the waves the host had already queued behind it (a batch of waves runs between
two status reads) processed "records" past the log array -- garbage element indices, an illegal memory access. Every
wave kernel now bounds its range by the window (gen_limit, zb_kernels.hpp); the step fails with ZB_ENOMEM.
"""
import os
import subprocess
import sys

import msgpack
import pytest

from test_gpu_long_running import Driver, _job_events
from zeebe_amd import records as R, workloads

pytestmark = pytest.mark.gpu


def _create_and_cancel_in_one_wave():
    c1, c4t = workloads.CONFIGS["c1"], workloads.CONFIGS["c4twin"]
    d = Driver({100: c1["workflow"]().to_xml(), 200: c4t["workflow"]().to_xml()},
               log_capacity=4096, row_capacity=1024, arena_bytes=2 << 20)
    pay = lambda b, n: [msgpack.packb({"orderId": b + i}) for i in range(n)]  # noqa: E731
    # tick 0: instances that end up waiting on jobs, some inside a subprocess (a scope with a live child)
    d.tick([("process", pay(0, 6)), ("subs", pay(10, 6))], [], [])
    roots = sorted(k for k, parent, *_ in d.e.instances() if parent == -1)
    for t in range(1, 4):
        # new CREATEs next to CANCELs: the CANCELs' TERMINATING events share a wave with the CREATED events
        cancels = [(R.RT_COMMAND, R.VT_WORKFLOW_INSTANCE, R.WI_CANCEL, wik, b"\x80") for wik in roots[:2]]
        roots = roots[2:]
        d.pending = [(k, r) for k, r in d.pending
                     if msgpack.unpackb(r.value, raw=False)["headers"]["workflowInstanceKey"] in roots]
        done, d.pending = d.pending[:2], d.pending[2:]
        d.tick([("subs", pay(100 * t, 8)), ("process", pay(100 * t + 50, 8))], _job_events(done, t), cancels)
        roots = sorted(k for k, parent, *_ in d.e.instances() if parent == -1)
    assert d.e.counters()["canceled"] == 6
    d.e.close()


def test_create_and_cancel_in_one_wave():
    _create_and_cancel_in_one_wave()


def test_create_and_cancel_in_one_wave_guard_bands():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ZB_CHECKED_LIBRARY="1", PYTHONPATH=os.pathsep.join([root, os.path.join(root, "tests")]))
    code = ("import test_gpu_regressions as t; from zeebe_amd.engine import checked_violations; "
            "t._create_and_cancel_in_one_wave(); assert checked_violations()[0] == 0; print('regression ok')")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "regression ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def test_log_overflow_mid_tick_fails_cleanly():
    from zeebe_amd import bpmn
    from zeebe_amd.engine import Engine, ZbError

    n = 600_000  # 9 records per instance: 5.4M records into a 4.8M-record log, several waves after the overflow
    wf = bpmn.Bpmn.create_executable_process("p").start_event("s").end_event("e").done()
    e = Engine(wave_only=True, log_capacity=n * 8, row_capacity=n * 3, arena_bytes=n * 256 + (64 << 20))
    e.deploy(wf.to_xml(), 100, 1)
    blob, offs = workloads.order_payloads(n)
    e.create_packed("p", blob, offs)
    with pytest.raises(ZbError) as ex:
        e.step()
    assert ex.value.code == -2 and "log-capacity" in str(ex.value), ex.value
    e.close()
    # the device is usable afterwards: the same tick in a log that holds it
    e = Engine(wave_only=True, log_capacity=n * 10, row_capacity=n * 3, arena_bytes=n * 256 + (64 << 20))
    e.deploy(wf.to_xml(), 100, 1)
    e.create_packed("p", blob, offs)
    st = e.step()
    assert st["quiescent"] and st["completed_instances"] == n and e.log_size() == 9 * n, st
    e.close()


def test_arena_overflow_mid_tick_fails_cleanly():
    # the merge results of the canonical job harness outgrow the arena in the middle of the tick: the wave that
    # overflows counts merge jobs it could not reserve (their list entries unwritten); k_merge / k_cond of that wave
    # and every later one skip their lists once a device error is flagged (wave_void, zb_kernels.hpp)
    from zeebe_amd import bpmn
    from zeebe_amd.engine import Engine, ZbError

    n = 200_000
    wf = bpmn.chain_workflow(4)
    jp = {"t%d" % k: msgpack.packb({"k%d" % k: "v" * (8 * k)}) for k in range(1, 5)}
    blob, offs = workloads.order_payloads(n)

    def run(arena):
        e = Engine(wave_only=True, log_capacity=n * 48, row_capacity=n * 8, arena_bytes=arena)  # (42 records per instance)
        e.deploy(wf.to_xml(), 100, 1)
        for act, p in jp.items():
            e.set_job_payload(100, act, p)
        e.create_packed("chain", blob, offs)
        return e

    e = run(24 << 20)  # (the CREATE payloads take ~3 MB; the four merges per instance ~40 MB)
    with pytest.raises(ZbError) as ex:
        e.step()
    assert ex.value.code == -2 and "arena-capacity" in str(ex.value), ex.value
    e.close()
    e = run(n * 512 + (64 << 20))
    st = e.step()
    assert st["quiescent"] and st["completed_instances"] == n, st
    e.close()
