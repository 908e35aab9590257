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

Partitions are exchanged as fixed 256-byte records (`zb_exchange_rec` in include/zb_engine.h),
so one `all_to_all_single` over RCCL (backend "nccl", xGMI) moves a whole round for every rank
(`DistCluster`); `LocalCluster` runs several partitions in one process (tests, single GPU).
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence

import numpy as np

REC_BYTES = 256
KIND_OPEN = 1
KIND_CORRELATE = 2
NAME_MAX, CK_MAX, PAYLOAD_MAX = 48, 48, 112
NO_TOKEN = 0xFFFFFFFF

# int32 kind, target, wf_partition; u32 token; i64 wik, aik, source_position; u16 elem; u8 name_len, ck_len;
# u16 payload_len, pad; name[48] ck[48] payload[112]
_HDR = struct.Struct("<iiiIqqqHBBHH")
assert _HDR.size == 48


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


def pack(records: Sequence[dict]) -> np.ndarray:
    """dicts (kind, partition, wf_partition, wik, aik, name, ck, payload[, token, elem, source_position])
    -> uint8 array of len * 256."""
    out = np.zeros(len(records) * REC_BYTES, dtype=np.uint8)
    for i, r in enumerate(records):
        name, ck, payload = r["name"], r.get("ck", b""), r.get("payload", b"")
        if len(name) > NAME_MAX or len(ck) > CK_MAX or len(payload) > PAYLOAD_MAX:
            raise ValueError("exchange record field too long (name <= 48, correlation key <= 48, payload <= 112 B)")
        hdr = _HDR.pack(r["kind"], r["partition"], r.get("wf_partition", 0), r.get("token", NO_TOKEN), r["wik"],
                        r["aik"], r.get("source_position", -1), r.get("elem", 0xFFFF), len(name), len(ck),
                        len(payload), 0)
        row = hdr + name.ljust(NAME_MAX, b"\0") + ck.ljust(CK_MAX, b"\0") + payload.ljust(PAYLOAD_MAX, b"\0")
        out[i * REC_BYTES:(i + 1) * REC_BYTES] = np.frombuffer(row, dtype=np.uint8)
    return out


def unpack(buf) -> List[dict]:
    b = bytes(np.asarray(buf, dtype=np.uint8))
    out = []
    for i in range(len(b) // REC_BYTES):
        row = b[i * REC_BYTES:(i + 1) * REC_BYTES]
        kind, tgt, wfp, token, wik, aik, spos, elem, nl, cl, pl, _ = _HDR.unpack_from(row)
        o = 48
        out.append(dict(kind=kind, partition=tgt, wf_partition=wfp, token=token, wik=wik, aik=aik,
                        source_position=spos, elem=elem, name=row[o:o + nl], ck=row[o + 48:o + 48 + cl],
                        payload=row[o + 96:o + 96 + pl]))
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
            for buf, counts in boxes:
                off = int(sum(counts[:q]))
                n = int(counts[q])
                if n:
                    pieces.append(buf[off * REC_BYTES:(off + n) * REC_BYTES])
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

    Each round: an all_reduce of the pending counts decides the step; an exchange is one
    all_to_all_single of the per-target counts and one all_to_all_single of the 256-byte records
    (RCCL over xGMI with backend "nccl" and device buffers; gloo with host buffers in the CPU tests).
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
        if self.rccl:
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

        buf, counts = self.p.outbox(kind)
        send_counts = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=self.device)
        recv_counts = torch.empty_like(send_counts)
        self.dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        rc = [int(x) for x in recv_counts.tolist()]
        sc = [int(x) for x in counts]
        send = self._tensor(buf).to(torch.uint8).contiguous()
        recv = torch.empty(sum(rc) * REC_BYTES, dtype=torch.uint8, device=self.device)
        self.dist.all_to_all_single(recv, send, [c * REC_BYTES for c in rc], [c * REC_BYTES for c in sc],
                                    group=self.group)
        if sum(rc):
            self.p.inbox(kind, recv)

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
