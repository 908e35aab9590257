"""Multi-partition stepping with message correlation.

A topic has P partitions; each has its own log, key generators and state, and instances never
migrate. The only traffic between partitions is message correlation
(`SubscriptionCommandSender.java:83-128`):

  * an open-subscription command, sent by the workflow partition when a message catch event is
    activated (`SubscribeMessageHandler.java:77-141`) to partition `abs(javaHash(ck) % P)`
    (`SubscriptionCommandSender.java:105-109`, `SubscriptionUtil.java:30-38`);
  * a correlate command, sent by the message partition when a published message meets a
    subscription (`PublishMessageProcessor.java:107-124`, `OpenMessageSubscriptionProcessor.java:85-92`)
    back to the workflow instance's partition.

The reference sends these over TCP whenever a side effect runs, so their arrival order is timing
dependent. Here they follow one canonical schedule that the GPU engines and the oracle both obey:

    repeat: run every partition to quiescence;
            if any partition holds open-subscription commands: deliver all of them, continue;
            if any partition holds correlate commands: deliver all of them, continue;
            stop.

A delivery appends, on each target partition, the commands of source partition 0, then 1, ...,
each source's in the order its processors produced them (log order of the records that produced
them). Messages are published at a point of quiescence, routed by the same hash.

Partitions exchange commands as batches (`zb_exchange_rec` in include/zb_engine.h): per (source, target) pair
one contiguous block [count][total bytes][count 64-byte headers][variable bytes: name, correlation key, payload],
so names, correlation keys and payloads have no length limit. GPU engines exchange their device-resident
batches with grouped RCCL send / receive over xGMI (`DistCluster` with the engine's own communicator, the
engine's zb_comm_exchange); torch.distributed (gloo) carries only the RCCL unique id and the control decisions.
`LocalCluster` runs several partitions in one process (tests, single GPU).
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence

import numpy as np

KIND_OPEN = 1
KIND_CORRELATE = 2
NO_TOKEN = 0xFFFFFFFF
BATCH_HEADER = 16

# int32 kind, target, wf_partition; u32 token; i64 wik, aik, source_position; u16 elem, pad; u32 name_len,
# ck_len, payload_len; u64 var_offset
_HDR = struct.Struct("<iiiIqqqHHIIIQ")
assert _HDR.size == 64


def java_hash(b: bytes) -> int:
    """SubscriptionUtil.getSubscriptionHashCode: 31-hash over SIGNED bytes, int32 wraparound."""
    h = 0
    for x in b:
        h = (h * 31 + (x - 256 if x >= 128 else x)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def subscription_partition(correlation_key: bytes, partition_count: int) -> int:
    """abs(hash % P) with Java's remainder (sign of the dividend), SubscriptionCommandSender.java:105-109."""
    h = java_hash(correlation_key)
    r = abs(h) % partition_count
    return r


def pack_batch(records: Sequence[dict]) -> bytes:
    """One exchange batch of dicts (kind, partition, wf_partition, wik, aik, name[, ck, payload, token, elem,
    source_position])."""
    if not records:
        return b""
    hdrs, var = [], bytearray()
    for r in records:
        name, ck, payload = r["name"], r.get("ck", b""), r.get("payload", b"")
        hdrs.append(_HDR.pack(r["kind"], r["partition"], r.get("wf_partition", 0), r.get("token", NO_TOKEN), r["wik"],
                              r["aik"], r.get("source_position", -1), r.get("elem", 0xFFFF), 0, len(name), len(ck),
                              len(payload), len(var)))
        v = name + ck + payload
        var += v + b"\0" * (-len(v) % 8)
    body = b"".join(hdrs) + bytes(var)
    return struct.pack("<QQ", len(records), BATCH_HEADER + len(body)) + body


def pack(records: Sequence[dict], partition_count: int):
    """Records in emission order -> (uint8 array of one batch per target partition, back to back in target order,
    byte size of each target's batch)."""
    by = [[] for _ in range(partition_count)]
    for r in records:
        by[r["partition"]].append(r)
    parts = [pack_batch(b) for b in by]
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy(), [len(p) for p in parts]


def unpack(buf) -> List[dict]:
    """Every command of a sequence of exchange batches, in order."""
    b = bytes(np.asarray(buf, dtype=np.uint8))
    out, o = [], 0
    while o < len(b):
        n, total = struct.unpack_from("<QQ", b, o)
        var0 = o + BATCH_HEADER + 64 * n
        for j in range(n):
            kind, tgt, wfp, token, wik, aik, spos, elem, _, nl, cl, pl, vo = _HDR.unpack_from(b, o + BATCH_HEADER + 64 * j)
            v = var0 + vo
            out.append(dict(kind=kind, partition=tgt, wf_partition=wfp, token=token, wik=wik, aik=aik,
                            source_position=spos, elem=elem, name=b[v:v + nl], ck=b[v + nl:v + nl + cl],
                            payload=b[v + nl + cl:v + nl + cl + pl]))
        o += total
    return out


class LocalCluster:
    """P partitions in one process. A partition object provides:
    run(), pending(kind) -> int, outbox(kind) -> (uint8 buffer, counts per target partition),
    inbox(kind, buffer), publish(name, correlation_key, payload, ttl)."""

    def __init__(self, partitions: Sequence):
        self.parts = list(partitions)
        self.rounds = 0

    def _exchange(self, kind: int):
        P = len(self.parts)
        boxes = [p.outbox(kind) for p in self.parts]
        for q in range(P):
            pieces = []
            for buf, sizes in boxes:  # source order: the canonical delivery order
                off = int(sum(sizes[:q]))
                n = int(sizes[q])
                if n:
                    pieces.append(buf[off:off + n])
            if pieces:
                self.parts[q].inbox(kind, _concat(pieces))

    def settle(self, max_rounds: int = 10000):
        for _ in range(max_rounds):
            for p in self.parts:
                p.run()
            self.rounds += 1
            if any(p.pending(KIND_OPEN) for p in self.parts):
                self._exchange(KIND_OPEN)
                continue
            if any(p.pending(KIND_CORRELATE) for p in self.parts):
                self._exchange(KIND_CORRELATE)
                continue
            return
        raise RuntimeError("no quiescence after %d rounds" % max_rounds)

    def publish(self, name: bytes, correlation_keys: Sequence[bytes], payloads: Sequence[bytes],
                ttl: int = 3600000):
        """PUBLISH commands in the given order, each on partition abs(hash(ck) % P), then settle."""
        P = len(self.parts)
        by_part = [[] for _ in range(P)]
        for ck, pl in zip(correlation_keys, payloads):
            by_part[subscription_partition(ck, P)].append((ck, pl))
        for q, items in enumerate(by_part):
            if items:
                self.parts[q].publish(name, [c for c, _ in items], [p for _, p in items], ttl)
        self.settle()


def _concat(pieces):
    try:
        import torch

        if isinstance(pieces[0], torch.Tensor):
            return torch.cat(pieces)
    except ImportError:
        pass
    return np.concatenate(pieces)


class DistCluster:
    """One partition per rank of a torch.distributed process group (partition id = rank).

    GPU engines (rccl=True, the default for them): the engine's own RCCL communicator moves the batches
    (zb_comm_pending / zb_comm_exchange: grouped ncclSend / ncclRecv over xGMI, with a failure protocol);
    torch.distributed only broadcasts the RCCL unique id. Other partitions (the oracle, CPU tests): each round an
    all_reduce of the pending counts decides the step, and an exchange is one all_to_all_single of the per-target
    byte sizes and one of the batches (host buffers, gloo).
    """

    def __init__(self, partition, group=None, device=None, rccl=None):
        """rccl: exchange through the engine's own RCCL communicator (GPU engines: default), else through
        torch.distributed on host buffers (oracle partitions, gloo)."""
        import torch
        import torch.distributed as dist

        self.p = partition
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device if device is not None else torch.device("cpu")
        self.rounds = 0
        self.rccl = hasattr(partition, "comm_exchange") if rccl is None else rccl
        # (one partition with no collective to run: its exchange is a device-side delivery to itself, no communicator)
        needs = getattr(partition, "needs_communicator", lambda: True)()
        if self.rccl and needs:
            # the 128-byte RCCL id travels over the control plane; the data path is RCCL (xGMI)
            obj = [partition.comm_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            partition.comm_init(obj[0], self.world, self.rank)

    def _tensor(self, x):
        import torch

        if isinstance(x, torch.Tensor):
            return x.to(self.device)
        return torch.as_tensor(np.asarray(x), device=self.device)

    def _exchange(self, kind: int):
        import torch

        buf, sizes = self.p.outbox(kind)
        send_sizes = torch.tensor([int(c) for c in sizes], dtype=torch.int64, device=self.device)
        recv_sizes = torch.empty_like(send_sizes)
        self.dist.all_to_all_single(recv_sizes, send_sizes, group=self.group)
        rs = [int(x) for x in recv_sizes.tolist()]
        ss = [int(x) for x in sizes]
        send = self._tensor(buf).to(torch.uint8).contiguous()
        recv = torch.empty(sum(rs), dtype=torch.uint8, device=self.device)
        self.dist.all_to_all_single(recv, send, rs, ss, group=self.group)
        if sum(rs):
            self.p.inbox(kind, recv.cpu().numpy())

    def _any_pending(self, kind: int) -> bool:
        import torch

        t = torch.tensor([int(self.p.pending(kind))], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item()) > 0

    def settle(self, max_rounds: int = 10000):
        for _ in range(max_rounds):
            self.p.run()
            self.rounds += 1
            if self.rccl:
                g_open, g_corr = self.p.comm_pending()
                if g_open:
                    self.p.comm_exchange(KIND_OPEN)
                    continue
                if g_corr:
                    self.p.comm_exchange(KIND_CORRELATE)
                    continue
                return
            if self._any_pending(KIND_OPEN):
                self._exchange(KIND_OPEN)
                continue
            if self._any_pending(KIND_CORRELATE):
                self._exchange(KIND_CORRELATE)
                continue
            return
        raise RuntimeError("no quiescence after %d rounds" % max_rounds)

    def publish(self, name: bytes, correlation_keys: Sequence[bytes], payloads: Sequence[bytes],
                ttl: int = 3600000):
        """Every rank passes the same global message list; each publishes the ones routed to it."""
        mine = [(ck, pl) for ck, pl in zip(correlation_keys, payloads)
                if subscription_partition(ck, self.world) == self.rank]
        if mine:
            self.p.publish(name, [c for c, _ in mine], [p for _, p in mine], ttl)
        self.settle()
