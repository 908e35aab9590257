"""Measurement aid: wall time of each call of one C5 step (bench_extra.run_c5's step) on one rank."""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import msgpack  # noqa: E402
import numpy as np  # noqa: E402
from zeebe_amd.engine import Engine, lib  # noqa: E402

lib()  # (before torch: the engine's RCCL)
import torch.distributed as tdist  # noqa: E402

from zeebe_amd import bpmn, cluster  # noqa: E402

s = socket.socket(); s.bind(("127.0.0.1", 0))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", str(s.getsockname()[1])); s.close()
tdist.init_process_group("gloo", rank=0, world_size=1)
n = 1_000_000
eng = Engine(log_capacity=n * 24, row_capacity=4 * n + 1024, arena_bytes=n * 640 + (64 << 20))
eng.deploy(bpmn.message_workflow().to_xml(), 100, 1)
create_payloads = [msgpack.packb({"orderId": "order-%d" % i}) for i in range(n)]
cks = [b"order-%d" % i for i in range(n)]
paid = msgpack.packb({"paid": True})
ck_off = np.zeros(n + 1, dtype=np.uint64); ck_off[1:] = np.cumsum([len(c) for c in cks])
pl_off = np.arange(n + 1, dtype=np.uint64) * len(paid)
ck_blob, pl_blob = b"".join(cks), paid * n
dc = cluster.DistCluster(eng)
T = {}


def tm(name, f, *a):
    t = time.perf_counter(); r = f(*a); T[name] = T.get(name, 0) + time.perf_counter() - t; return r


orig_run, orig_pend, orig_xchg = eng.run, eng.comm_pending, eng.comm_exchange
eng.run = lambda: tm("run", orig_run)
eng.comm_pending = lambda: tm("comm_pending", orig_pend)
eng.comm_exchange = lambda k: tm("comm_exchange_%d" % k, orig_xchg, k)
for it in range(3):
    eng.reset(); eng.create("msg", create_payloads)
    T.clear(); t0 = time.perf_counter()
    tm("settle1", dc.settle)
    tm("publish", eng.publish_packed, b"order", ck_blob, ck_off, pl_blob, pl_off, 3600000)
    tm("settle2", dc.settle)
    tm("serialize", eng.serialize, 0, eng.log_size())
    print("step %.2f ms" % ((time.perf_counter() - t0) * 1e3), {k: round(v * 1e3, 2) for k, v in T.items()}, "rounds", dc.rounds)
tdist.destroy_process_group()
