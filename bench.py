"""bench.py — BPMN element transitions/s on MI355X (BASELINE.json metric), one partition per GPU.

Default workload (BASELINE.json configs[2], the largest single-GPU configuration and the one north_star's
">= 50 % of HBM roofline for 10M concurrent instances" target names): two exclusive
gateways with json-el conditions over msgpack payloads {"amount", "region", "score"} (Philox, seed 42),
10,000,000 concurrent instances per GPU. One step = one processing tick of the partition
(GPU timing):
  1. inject the staged 10M CREATE commands (resident in HBM) at the log tail,
  2. run every lockstep wave to quiescence (~101.7M records written, all WORKFLOW_INSTANCE events: 11 or 13
     transitions per instance),
  3. drain: serialize every record the tick wrote into the exact reference record values + record
     headers, in HBM (zb_serialize) -- the emitted record stream a JNI shim appends to the log.
The D2H copy of that stream into pinned host memory crosses PCIe; per the task contract it is never
`value` and is reported beside it (value_pcie_inclusive), measured on one extra step.

--config c2 | c3 | c4 | c5 selects another BASELINE configuration (c5: bench_extra.py).
Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process and one partition per GPU;
rank r takes the contiguous block of instances [r*n, (r+1)*n) of the node (instances are independent, so this
is the same per-partition load as the reference's round-robin dispatch; payloads are counter-based per
instance index, so every instance's payload is the same whatever the partitioning). Partitions never
communicate for C1-C4 (weak scaling, no data-path collective; barrier + max-over-ranks timing through
torch.distributed gloo).

Prints ONE JSON line on rank 0 with "roofline" and "cpu_baseline".
"""
import argparse
import json
import os
import platform
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BYTES_PER_TRANSITION = 96  # 32 B row read + 32 B row write + 32 B record descriptor
DESC_BYTES = 32  # one zb_rec descriptor per log record
HDR_BYTES = 24  # one zb_record_header per drained record
PMC_DIRS = [os.path.join(ROOT, "profiles", r) for r in ("r06", "r05", "r04", "r03")]  # newest first
METRIC = "BPMN element transitions/sec (+ completed instances/sec) per node; % HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=("c1", "c2", "c3", "c4", "c5"), default="c3")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instances", type=int, default=0, help="per GPU (default: C3 10,000,000, C2/C4/C5 1,000,000)")
    ap.add_argument("--tasks", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=0, help="instances in the 1-thread oracle sample (0: default)")
    ap.add_argument("--cpu-partitions", type=int, default=0, help="C5: oracle partitions (threads) of the CPU sample (0: 8)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the extra C2 wave-only / C4 lines")
    ap.add_argument("--no-drain", action="store_true", help="device stepping only (not the contract's step)")
    ap.add_argument("--wave-only", action="store_true", help="force the general wave pipeline (no trajectory path)")
    ap.add_argument("--jobs", choices=("harness", "external", "processor"), default=None,
                    help="job mode: the canonical in-kernel harness, ZB_CFG_EXTERNAL_JOBS or ZB_CFG_JOB_PROCESSOR (the "
                         "modes INTEGRATION.md binds). Default: external for C3 (no service task: the integration's "
                         "configuration), the harness for the configurations with service tasks (their bench ticks "
                         "complete jobs in-kernel)")
    ap.add_argument("--frames", action="store_true",
                    help="drain log frames (zb_serialize_frames, with request metadata on every CREATE) instead of "
                         "values + headers")
    ap.add_argument("--steady", action="store_true",
                    help="C2 steady state (bench_steady.py): live instances waiting on jobs, ticks of job completions, "
                         "creates and cancels, external job processor")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on GPU 0 (multi-rank rehearsal on a one-GPU box; not a scaling run)")
    a = ap.parse_args()
    if a.jobs is None:
        a.jobs = "external" if a.config == "c3" else "harness"
    if a.jobs != "harness" and a.config != "c3":
        ap.error("--jobs %s: only C3 (no service task) runs a tick to quiescence without a job processor" % a.jobs)
    return a


# ------------------------------------------------------------------------------ workloads
def workload(cfg, n, start, tasks=20):
    """(xml, process id, payload blob, offsets, job payloads, description) for instances [start, start + n)."""
    from zeebe_amd import bpmn, workloads

    if cfg == "c3":
        blob, offs = workloads.xor_payloads_np(n, start=start)
        return (bpmn.xor_workflow().to_xml(), "xor", blob, offs, {},
                "C3: exclusive gateways with json-el conditions over msgpack payloads, %d concurrent instances "
                "per GPU" % n)
    if cfg == "c1":
        blob, offs = workloads.order_payloads(n, start=start)
        return (bpmn.chain_workflow(1).to_xml(), "chain", blob, offs,
                {"t1": b"\x81" + workloads.mp_str("step") + workloads.mp_int(1)},
                "C1: start -> one service task -> end, %d instances, canonical job harness (BASELINE configs[0], "
                "the reference's CPU-runnable case)" % n)
    if cfg == "c2":
        blob, offs = workloads.order_payloads(n, start=start)
        jp = {"t%d" % k: b"\x81" + workloads.mp_str("step") + workloads.mp_int(k) for k in range(1, tasks + 1)}
        return (bpmn.chain_workflow(tasks).to_xml(), "chain", blob, offs, jp,
                "C2: %d-service-task chain, %d concurrent instances per GPU, canonical job harness, default "
                "output merges" % (tasks, n))
    if cfg == "c4":
        blob, offs = workloads.order_payloads(n, start=start)
        jp = {"task%d" % k: b"\x81" + workloads.mp_str("sub") + workloads.mp_int(k) for k in range(1, 9)}
        return (bpmn.parallel_workflow(8).to_xml(), "par", blob, offs, jp,
                "C4: parallel fork/join (fan-out 8) with embedded sub-process scopes, %d instances per GPU "
                "(EXTENSION, parity unpinned)" % n)
    raise ValueError(cfg)


RECS_PER_INST = {"c1": lambda t: 18, "c2": lambda t: 2 + 8 + 5 * t + 3 * t, "c3": lambda t: 16, "c4": lambda t: 200}


def make_engine(cfg, n, a, rank, world, local_rank):
    from zeebe_amd.engine import CFG_SHARED_GPU, Engine

    recs = RECS_PER_INST[cfg](a.tasks)
    # (the trajectory path allocates no rows for instances that complete in the tick; the wave pipeline holds a
    # row per live element instance: C3 wave-only needs the process + gateway / task rows of every instance)
    rows = {"c1": n * 3, "c2": n * (a.tasks + 2), "c3": n * 3 if a.wave_only else 1 << 20, "c4": n * 20}[cfg]
    arena = {"c1": n * 96, "c2": n * (48 + 48 * a.tasks), "c3": n * 64, "c4": n * 1200}[cfg] + (64 << 20)
    jobs = getattr(a, "jobs", "harness") if cfg == "c3" else "harness"  # (service tasks: the in-kernel harness)
    return Engine(device=0 if a.same_device else local_rank, partition_id=rank, partition_count=world,
                  log_capacity=int(n * recs), row_capacity=int(rows), arena_bytes=int(arena), wave_only=a.wave_only,
                  external_jobs=jobs == "external", job_processor=jobs == "processor",
                  flags=CFG_SHARED_GPU if a.same_device and world > 1 else 0)


FRAME_CFG = dict(stream_id=1, raft_term=3, timestamp=1_700_000_000_000)  # (the broker's log stream / raft term)


def run_workload(cfg, n, a, rank, world, local_rank, barrier, steps, warmup, drain=True, pcie=False):
    xml, pid, blob, offs, jp, desc = workload(cfg, n, rank * n, a.tasks)
    eng = make_engine(cfg, n, a, rank, world, local_rank)
    eng.deploy(xml, 100, 1)
    for act, p in jp.items():
        eng.set_job_payload(100, act, p)
    eng.create_packed(pid, blob, offs)
    create_bytes = len(blob) + 4 * n  # the CREATE payload documents ([u32 len][bytes]) in the arena
    del blob
    frames = getattr(a, "frames", False)
    if frames:  # every CREATE carries its client request (CreateWorkflowInstanceRequest: request id, stream id)
        import numpy as np

        eng.set_request_metadata_np(np.arange(n, dtype=np.uint64) + (rank << 40), np.arange(n, dtype=np.int32) % 64)
    eng.upload_staged()  # (the staged batch in HBM before the timed region)

    def one_step():
        eng.reset(keep_staged=True)
        t0 = time.perf_counter()
        st = eng.step()
        t1 = time.perf_counter()
        assert st["quiescent"], st
        ser = None
        if drain and frames:  # the tick's records as log frames (the broker appends them: INTEGRATION.md)
            ser = eng.serialize_frames(n, eng.log_size() - n, **FRAME_CFG)
        elif drain:  # the tick's emitted records (everything after the n injected commands)
            ser = eng.serialize(n, eng.log_size() - n)
        t2 = time.perf_counter()
        return st, ser, t1 - t0, t2 - t1

    for _ in range(warmup):
        one_step()
    barrier()
    tot = dict(transitions=0, completed=0, written=0, merges=0, merge_bytes=0, cond_bytes=0, kernel_ms=0.0,
               process_ms=0.0, emit_ms=0.0, aux_ms=0.0, main_ms=0.0, launches=0, waves=0, step_s=0.0, drain_s=0.0,
               ser_write_ms=0.0, ser_size_ms=0.0, value_bytes=0, payload_bytes=0, drained=0, path=0, generic_tiles=0,
               template_drain=0, create_bytes=0, instances=n)
    t0 = time.perf_counter()
    for _ in range(steps):
        st, ser, ts, td = one_step()
        tot["transitions"] += st["transitions"]
        tot["completed"] += st["completed_instances"]
        tot["written"] += st["records_written"]
        tot["merges"] += st["merges"]
        tot["merge_bytes"] += st["merge_bytes"]
        tot["cond_bytes"] += st["condition_payload_bytes"]
        tot["kernel_ms"] += st["wave_kernel_ms"]
        tot["process_ms"] += st["process_kernel_ms"]
        tot["emit_ms"] += st["emit_kernel_ms"]
        tot["aux_ms"] += st["aux_kernel_ms"]
        tot["main_ms"] += st["main_emit_kernel_ms"]
        tot["launches"] += st["launches"]
        tot["waves"] += st["waves"]
        tot["path"] = st["path"]
        tot["step_s"] += ts
        tot["drain_s"] += td
        if ser:
            tot["ser_write_ms"] += ser["write_kernel_ms"]
            tot["ser_size_ms"] += ser["size_kernel_ms"]
            tot["value_bytes"] += ser["value_bytes"]
            tot["payload_bytes"] += ser["payload_bytes"]
            tot["drained"] += ser["records"]
            tot["generic_tiles"] += ser["generic_tiles"]
            tot["template_drain"] += ser["template_drain"]
    barrier()
    tot["elapsed"] = time.perf_counter() - t0
    tot["desc"] = desc
    tot["create_bytes"] = create_bytes
    tot["frames"] = frames
    tot["jobs"] = getattr(a, "jobs", "harness") if cfg == "c3" else "harness"
    tot["desc"] += {"harness": ", canonical job harness", "external": ", ZB_CFG_EXTERNAL_JOBS (the integration's job mode)",
                    "processor": ", ZB_CFG_JOB_PROCESSOR"}[tot["jobs"]] if cfg == "c3" else ""
    if pcie and drain:
        tot["pcie"] = pcie_step(eng, n, one_step)
    eng.close()
    return tot


def pcie_step(eng, n, one_step, chunk=256 << 20):
    """One more tick with the drained stream copied to pinned host memory in 256 MiB chunks (double
    buffered host-side; each chunk is consumed before its buffer is reused)."""
    from zeebe_amd.engine import pinned_alloc, pinned_free

    bufs = [pinned_alloc(chunk), pinned_alloc(chunk)]
    try:
        t0 = time.perf_counter()
        st, ser, _, _ = one_step()
        t1 = time.perf_counter()
        total, off, k = ser["value_bytes"], 0, 0
        while off < total:
            m = min(chunk, total - off)
            eng.drain_copy(bufs[k & 1], off, m)
            off += m
            k += 1
        t2 = time.perf_counter()
    finally:
        for b in bufs:
            pinned_free(b)
    return {"transitions": st["transitions"], "tick_s": t1 - t0, "d2h_s": t2 - t1, "bytes": ser["value_bytes"],
            "d2h_GBps": ser["value_bytes"] / (t2 - t1) / 1e9 if t2 > t1 else 0.0}


# ------------------------------------------------------------------------------ CPU baseline
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _oracle_partition(cfg, n, start, tasks):
    from oracle import zbref

    xml, pid, blob, offs, jp, _ = workload(cfg, n, start, tasks)
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    for act, p in jp.items():
        o.set_job_payload(100, act, p)
    o.create_packed(pid, blob, offs)
    return o


def _partition_proc(cfg, per, i, tasks, barrier, q):
    """One oracle partition in its own process (forked before the GPU is touched): built, warmed, run at the
    barrier; reports (records, transitions, completed, instances, t0, t1)."""
    import ctypes

    w = _oracle_partition(cfg, per, i * per, tasks)  # untimed warm-up: faults in the process's heap
    w._L.zbref_run_timed(w._h, ctypes.byref(ctypes.c_int64()))
    w.close()
    o = _oracle_partition(cfg, per, i * per, tasks)
    nrec = ctypes.c_int64()
    barrier.wait()
    t0 = time.perf_counter()
    o._L.zbref_run_timed(o._h, ctypes.byref(nrec))
    t1 = time.perf_counter()
    c = o.counters()
    q.put((nrec.value, c["transitions"], c["completed"], c["created"], t0, t1))


def cpu_baseline_line(cfg, tasks, sample):
    """The oracle (sequential C++ restatement of the reference path, same canonical schedule) on a bounded
    sample of the same workload: 1 partition on 1 core, and P = min(8, cores) partitions on P cores, one process
    per partition (the reference runs one stream processor per partition; a process each keeps the restatement's
    allocations per partition, as a JVM's thread-local allocation buffers do -- threads sharing one C heap scaled
    4.7x on 8 cores, processes scale with the cores). Run from a process forked before the GPU is
    initialised (main)."""
    import multiprocessing as mp

    ctx = mp.get_context("fork")
    threads = min(8, os.cpu_count() or 1)
    res = {}
    for k in sorted({1, threads}):
        per = sample if k == 1 else max(sample // 2, 1)
        barrier, q = ctx.Barrier(k), ctx.Queue()
        ps = [ctx.Process(target=_partition_proc, args=(cfg, per, i, tasks, barrier, q)) for i in range(k)]
        for p in ps:
            p.start()
        out = [q.get() for _ in ps]
        for p in ps:
            p.join()
        wall = max(r[5] for r in out) - min(r[4] for r in out)
        res[k] = dict(records=sum(r[0] for r in out), transitions=sum(r[1] for r in out),
                      completed=sum(r[2] for r in out), instances=sum(r[3] for r in out), wall_s=wall)
    one, many = res[1], res[threads]
    return {"value": one["transitions"] / one["wall_s"], "unit": "transitions/s", "cores": 1, "kind": "port",
            "sample": "%s workload, %d instances (%d records processed) run to quiescence by oracle/zbref, 1 thread, "
                      "sequential FIFO, canonical job harness: %.2f s" % (cfg.upper(), one["instances"],
                                                                          one["records"], one["wall_s"]),
            "cpu_model": cpu_model(),
            "completed_instances_per_s": one["completed"] / one["wall_s"],
            "multi_partition": {"value": many["transitions"] / many["wall_s"], "cores": threads,
                                "partitions": threads, "instances": many["instances"], "wall_s": many["wall_s"],
                                "completed_instances_per_s": many["completed"] / many["wall_s"],
                                "scaling_vs_1": (many["transitions"] / many["wall_s"]) /
                                                (one["transitions"] / one["wall_s"]),
                                "note": "one oracle partition per process, run concurrently (SURVEY §8d: P "
                                        "partitions on P cores, P = min(8, cores))"}}


def cpu_baseline_early(a, rank, world):
    """cpu_baseline_line in a child forked before anything touches the GPU (its partitions fork in turn)."""
    if rank != 0 or world != 1 or a.no_cpu_baseline or a.config == "c5" or a.steady:
        return None
    import multiprocessing as mp

    sample = a.cpu_sample or {"c1": 10_000, "c3": 400_000, "c2": 30_000, "c4": 20_000}[a.config]
    ctx = mp.get_context("fork")
    q = ctx.Queue()

    def run():
        q.put(cpu_baseline_line(a.config, a.tasks, sample))

    p = ctx.Process(target=run)
    p.start()
    r = q.get()
    p.join()
    return r


# ------------------------------------------------------------------------------ roofline
def _pmc_file(tag):
    for d in PMC_DIRS:
        f = os.path.join(d, "pmc_%s.json" % tag)
        if os.path.exists(f):
            return f
    return None


def load_traffic(tag, kernel_prefix):
    f = _pmc_file(tag)
    if f is None:
        return None, None
    with open(f) as fh:
        d = json.load(fh)
    for k, v in d.get("kernels", {}).items():
        if kernel_prefix in k and "hbm_bytes" in v:
            return v["hbm_bytes"], k
    return None, None


def load_traffic_step(tag, kernel_prefixes):
    """HBM bytes per tick of every kernel named by the prefixes (PMC averages x dispatches / ticks of the PMC run;
    the run's ticks = k_inject dispatches, one per tick)."""
    f = _pmc_file(tag)
    if f is None:
        return None
    with open(f) as fh:
        d = json.load(fh).get("kernels", {})
    ticks = sum(v.get("dispatches", 0) for k, v in d.items() if "k_inject" in k)
    if not ticks:
        return None
    tot = sum(v["hbm_bytes"] * v.get("dispatches", 0) for k, v in d.items()
              if "hbm_bytes" in v and any(k.startswith(p) or k.startswith("void " + p) for p in kernel_prefixes))
    return tot / ticks


def roofline(tot, steps, cfg, n):
    """Dominant kernel of the step: the drain's write pass or the main emit launch, by device time."""
    cands = []
    if tot["ser_write_ms"] > 0 and tot["template_drain"] == steps and tot.get("frames"):
        # the template drain writing log frames: every drained record's frame (104-byte prefix + value + padding)
        # written, per instance its CREATE descriptor, CREATE payload document and request metadata (24 B) read once
        b = (tot["value_bytes"] + steps * (tot["instances"] * (DESC_BYTES + 24) + tot["create_bytes"])) / steps
        cands.append(("zbg::k_tdrain_write<frames>", tot["ser_write_ms"] / steps, b,
                      "log frame bytes written per drained record (104 B prefix + value + padding) + 32 B CREATE "
                      "descriptor, the CREATE payload document and 24 B of request metadata read per instance"))
    elif tot["ser_write_ms"] > 0 and tot["template_drain"] == steps:
        # the template drain (zb_tdrain.hip): per launch every drained record's header and value written, and per
        # instance its CREATE descriptor and CREATE payload document read once (the traces and generation bases
        # are a few KB, read from the scalar cache)
        b = (tot["drained"] * HDR_BYTES + tot["value_bytes"] + steps * (tot["instances"] * DESC_BYTES +
                                                                          tot["create_bytes"])) / steps
        cands.append(("zbg::k_tdrain_write", tot["ser_write_ms"] / steps, b,
                      "24 B header + value bytes written per drained record + 32 B CREATE descriptor and the CREATE "
                      "payload document read per instance"))
    elif tot["ser_write_ms"] > 0:
        # per launch: every drained record's descriptor read + header write, its value bytes written and the
        # payload documents copied into them read (SURVEY §8d payload term)
        b = (tot["drained"] * (DESC_BYTES + HDR_BYTES) + tot["value_bytes"] + tot["payload_bytes"]) / steps
        # the wave-parallel fast write pass (k_ser_write over the tiles it leaves, if any) / single pass
        kname = ("zbg::k_ser_wave" if tot["generic_tiles"] == 0 else "zbg::k_ser_wave (+ k_ser_write on %d tiles)"
                 % (tot["generic_tiles"] // steps)) if tot["ser_size_ms"] > 0 else "zbg::k_ser_fused"
        cands.append((kname, tot["ser_write_ms"] / steps, b,
                      "32 B descriptor read + 24 B header write per drained record + value bytes written + payload "
                      "bytes read"))
    if tot["main_ms"] > 0 and tot["template_drain"] != steps:  # (a deferred batch writes no descriptors)
        b = (DESC_BYTES * tot["written"] + tot["merge_bytes"] + tot["cond_bytes"]) / steps
        kname = {1: "zbg::k_tmpl<false, false>", 2: "zbg::k_tmpl<true, false>"}.get(tot["path"], "zbg::k_tmpl")
        cands.append((kname, tot["main_ms"] / steps, b,
                      "32 B descriptor per record written + merge (job + scope + result) bytes + condition payload "
                      "bytes (the launch writes no element-instance rows per transition)"))
    if tot["path"] == 0 and tot["process_ms"] > 0:
        b = (BYTES_PER_TRANSITION * tot["transitions"] + tot["merge_bytes"] + tot["cond_bytes"]) / steps
        cands.append(("zbg::k_wave (fused process / scan / emit, + k_merge / k_cond / k_subscribe: every wave kernel)",
                      tot["kernel_ms"] / steps, b,
                      "SURVEY §8d: 96 B per transition + merge + condition bytes over all wave kernels of the step"))
    name, ms, b, model = max(cands, key=lambda c: c[1])
    achieved = b / (ms / 1e3) / 1e9
    if name.startswith("zbg::k_wave "):  # every wave kernel of the tick: their PMC bytes per tick
        traffic = load_traffic_step("%s_%d" % (cfg, n), ("zbg::k_wave", "zbg::k_merge", "zbg::k_cond",
                                                         "zbg::k_subscribe", "zbg::k_pre", "zbg::k_children"))
        pmc_kernel = "the wave kernels (per tick)"
    else:
        traffic, pmc_kernel = load_traffic("%s_%d" % (cfg, n), name.split(" ")[0].split("<")[0])
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": name, "avg_launch_us": ms * 1e3, "alg_bytes_per_launch": b,
         "alg_bytes_model": model,
         "traffic_note": ("HBM bytes per launch of %s from rocprofv3 FETCH_SIZE x2 + WRITE_SIZE (separate --pmc "
                          "passes, %s)" % (pmc_kernel, os.path.relpath(_pmc_file("%s_%d" % (cfg, n)), ROOT)))
                         if traffic else
                         "no committed PMC passes for this workload"}
    r["other_kernels"] = [{"kernel": c[0], "avg_launch_us": c[1] * 1e3, "alg_bytes_per_launch": c[2],
                           "achieved": c[2] / (c[1] / 1e3) / 1e9, "frac": c[2] / (c[1] / 1e3) / 1e9 / HBM_PEAK_GBS}
                          for c in cands if c[0] != name]
    # BASELINE.md §3 / SURVEY §8d: the whole path priced by its algorithmic bytes -- 96 B per transition + the
    # payload terms (merges, condition payloads) -- over the step's wall time (drain included)
    if tot.get("elapsed"):
        pb = (BYTES_PER_TRANSITION * tot["transitions"] + tot["merge_bytes"] + tot["cond_bytes"]) / steps
        pa = pb / (tot["elapsed"] / steps) / 1e9
        r["path_bytes_per_step"] = pb
        r["path_achieved"] = pa
        r["path_frac"] = pa / HBM_PEAK_GBS
        r["path_note"] = ("BASELINE.md §3: (96 B x transitions + merge + condition payload bytes) / step wall time / "
                          "8 TB/s; the step also writes the serialized record stream, which this model does not price")
    return r


# ------------------------------------------------------------------------------ main
def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.instances == 0:
        a.instances = {"c3": 10_000_000, "c1": 10_000}.get(a.config, 1_000_000)
    cpu_line = cpu_baseline_early(a, rank, world)  # (forks: before the GPU is initialised)
    # Load libzbgpu.so before torch: its DT_NEEDED HIP runtime and RCCL (/opt/rocm/lib) are then the copies the
    # process binds, so the engine's communicator runs on the system RCCL, not the one torch bundles
    # (zb_rccl_library reports the file; C5 prints it).
    from zeebe_amd.engine import lib

    lib()
    dist = None
    if world > 1:
        import torch.distributed as dist

        # Control plane only (barrier, max-over-ranks, sums): C1-C4 partitions never exchange data (weak
        # scaling, no data-path collective). gloo keeps torch's own HIP runtime out of the process: the engine
        # (libzbgpu.so) drives its GPU through the system ROCm runtime.
        dist.init_process_group("gloo")
    if a.config == "c5":
        return run_c5(a, rank, world, local_rank, dist)

    def barrier():
        if dist is not None:
            dist.barrier()

    def reduce(v, op):
        if dist is None:
            return v
        import torch

        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t.item())

    n = a.instances
    if a.steady:
        return run_steady_line(a, rank, world, local_rank, dist, barrier, reduce)
    tot = run_workload(a.config, n, a, rank, world, local_rank, barrier, a.steps, a.warmup, drain=not a.no_drain,
                       pcie=(rank == 0 and world == 1 and not a.no_drain))
    elapsed = tot["elapsed"]
    all_tr, all_comp = tot["transitions"], tot["completed"]
    if dist is not None:
        elapsed = reduce(elapsed, dist.ReduceOp.MAX)
        all_tr = reduce(all_tr, dist.ReduceOp.SUM)
        all_comp = reduce(all_comp, dist.ReduceOp.SUM)
    if rank == 0:
        steps = a.steps
        out = {
            "metric": METRIC,
            "value": all_tr / elapsed,
            "unit": "transitions/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed * 1e3 / steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (SURVEY §8d %s inputs, deterministic)" % a.config.upper(),
            "config": {"workload": tot["desc"], "instances_per_gpu": n, "partitions": world,
                       "parallelism": "partition-per-gpu", "jobs": a.jobs,
                       "timed_step": "inject staged CREATEs (in HBM) + lockstep waves to quiescence" +
                                     ("" if a.no_drain else
                                      " + zb_serialize_frames of every emitted record (log frames, in HBM)" if a.frames
                                      else " + zb_serialize of every emitted record (values + headers, in HBM)")},
            "completed_instances_per_s": all_comp / elapsed,
            "records_written_per_step": tot["written"] / steps,
            "wave_launches_per_step": tot["launches"] / steps,
            "step_breakdown_ms": {"stepping": tot["step_s"] * 1e3 / steps, "drain": tot["drain_s"] * 1e3 / steps,
                                  "stepping_kernels": tot["kernel_ms"] / steps,
                                  "drain_size_kernel": tot["ser_size_ms"] / steps,
                                  "drain_write_kernel": tot["ser_write_ms"] / steps},
            "value_stepping_only": tot["transitions"] / tot["step_s"] if tot["step_s"] else None,
            "drained_bytes_per_step": tot["value_bytes"] / steps + (0 if a.frames else HDR_BYTES * tot["drained"] / steps),
            "roofline": roofline(tot, steps, a.config, n),
        }
        if "pcie" in tot:
            p = tot["pcie"]
            out["value_pcie_inclusive"] = p["transitions"] / (p["tick_s"] + p["d2h_s"])
            out["pcie"] = {"d2h_GBps": p["d2h_GBps"], "bytes": p["bytes"], "tick_ms": p["tick_s"] * 1e3,
                           "d2h_ms": p["d2h_s"] * 1e3,
                           "note": "one extra tick whose drained values are copied to pinned host memory (256 MiB "
                                   "chunks); PCIe-inclusive rate, never `value` (task contract)"}
        if world == 1 and not a.no_extras and a.config == "c3":
            out["extras"] = extras(a, barrier)
        if cpu_line is not None:
            out["cpu_baseline"] = cpu_line
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def steady_line(t, steps, live):
    return {"value": t["transitions"] / t["elapsed"], "ms_per_step": t["elapsed"] * 1e3 / steps,
            "stepping_ms": t["step_s"] * 1e3 / steps, "drain_ms": t["drain_s"] * 1e3 / steps,
            "completed_instances_per_s": t["completed"] / t["elapsed"],
            "per_tick": {"input_records": t["inputs"] / steps, "job_completions": t["completions"] / steps,
                         "creates": t["creates"] / steps, "cancels": t["cancels"] / steps,
                         "records_written": t["written"] / steps, "transitions": t["transitions"] / steps,
                         "merges": t["merges"] / steps},
            "live_element_instances": t["live_rows"], "pending_jobs": t["pending_jobs"],
            "compactions": t["compactions"],
            "tick_ms_median": sorted(t["tick_ms"])[len(t["tick_ms"]) // 2] if t.get("tick_ms") else None,
            "tick_ms_max": max(t["tick_ms"]) if t.get("tick_ms") else None,
            "roofline": roofline(t, steps, "c2s", live), "workload": t["desc"]}


def run_steady_line(a, rank, world, local_rank, dist, barrier, reduce):
    import bench_steady

    live = a.instances
    t = bench_steady.run_steady(a, rank, world, local_rank, barrier, a.steps, a.warmup, live=live)
    elapsed, all_tr, all_comp = t["elapsed"], t["transitions"], t["completed"]
    if dist is not None:
        elapsed = reduce(elapsed, dist.ReduceOp.MAX)
        all_tr = reduce(all_tr, dist.ReduceOp.SUM)
        all_comp = reduce(all_comp, dist.ReduceOp.SUM)
    if rank == 0:
        line = steady_line(t, a.steps, live)
        out = {"metric": METRIC, "value": all_tr / elapsed, "unit": "transitions/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed * 1e3 / a.steps,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
               "data": "synthetic (C2 chain, steady-state job completion schedule, deterministic)",
               "config": {"workload": t["desc"], "live_instances_per_gpu": live, "partitions": world,
                          "parallelism": "partition-per-gpu",
                          "timed_step": "lockstep waves of one tick to quiescence (staged input already in HBM) + "
                                        "zb_serialize of every record the tick wrote"},
               "completed_instances_per_s": all_comp / elapsed}
        out.update({k: v for k, v in line.items() if k not in ("value", "ms_per_step", "workload")})
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = bench_steady.cpu_baseline_steady(40_000, 20)
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def extras(a, barrier):
    """Shorter lines on the other single-GPU configurations (same step definition, 3 steps each)."""
    out = {}
    import copy

    # the integration's own configuration (ZB_CFG_EXTERNAL_JOBS; the broker appends log frames through
    # LogStreamBatchWriter): C3 10M with values + headers, and with log frames carrying every CREATE's request metadata
    for name, frames in (("c3_integration_values", False), ("c3_integration_frames", True)):
        b = copy.copy(a)
        b.jobs, b.frames, b.wave_only = "external", frames, False
        t = run_workload("c3", 10_000_000, b, 0, 1, 0, barrier, 3, 1)
        out[name] = {"value": t["transitions"] / t["elapsed"], "ms_per_step": t["elapsed"] * 1e3 / 3,
                     "stepping_ms": t["step_s"] * 1e3 / 3, "drain_ms": t["drain_s"] * 1e3 / 3,
                     "path": t["path"], "template_drain": t["template_drain"] == 3,
                     "drained_bytes_per_step": t["value_bytes"] / 3 + (0 if frames else HDR_BYTES * t["drained"] / 3),
                     "roofline": roofline(t, 3, "c3f" if frames else "c3x", 10_000_000),
                     "workload": t["desc"] + ", ZB_CFG_EXTERNAL_JOBS, drain: " +
                                 ("log frames (zb_serialize_frames, request metadata on every CREATE)" if frames else
                                  "values + 24-byte headers (zb_serialize)")}

    b = copy.copy(a)
    b.wave_only = True
    t = run_workload("c2", 1_000_000, b, 0, 1, 0, barrier, 3, 1)
    out["c2_wave_only"] = {"value": t["transitions"] / t["elapsed"], "ms_per_step": t["elapsed"] * 1e3 / 3,
                           "stepping_ms": t["step_s"] * 1e3 / 3, "drain_ms": t["drain_s"] * 1e3 / 3,
                           "roofline": roofline(t, 3, "c2w", 1_000_000), "workload": t["desc"] + " (wave pipeline)"}
    t = run_workload("c3", 10_000_000, b, 0, 1, 0, barrier, 3, 1)
    out["c3_wave_only"] = {"value": t["transitions"] / t["elapsed"], "ms_per_step": t["elapsed"] * 1e3 / 3,
                           "stepping_ms": t["step_s"] * 1e3 / 3, "drain_ms": t["drain_s"] * 1e3 / 3,
                           "roofline": roofline(t, 3, "c3w", 10_000_000),
                           "workload": t["desc"] + " (general wave pipeline, no trajectory path)"}
    import bench_steady

    # (24 ticks: the partition compacts about every fifth tick, and the line's average carries its share)
    t = bench_steady.run_steady(a, 0, 1, 0, barrier, 24, 1, live=1_000_000)
    out["c2_steady"] = steady_line(t, 24, 1_000_000)
    out["c1_exact_tree"] = run_exact_tree(a)
    t = run_workload("c4", 1_000_000, a, 0, 1, 0, barrier, 3, 1)
    out["c4"] = {"value": t["transitions"] / t["elapsed"], "ms_per_step": t["elapsed"] * 1e3 / 3,
                 "stepping_ms": t["step_s"] * 1e3 / 3, "drain_ms": t["drain_s"] * 1e3 / 3,
                 "roofline": roofline(t, 3, "c4", 1_000_000), "workload": t["desc"]}
    return out


def run_exact_tree(a, n=1_000_000, steps=3):
    """The exact payload tree under load (zb_xmerge.hpp): C1 (start -> service task -> end), n instances whose job
    completion payload has a duplicate key, so every default output merge is one the structural merge refuses and the
    reference's own tree takes (MsgPackDocumentIndexer keeps the first position and the last value). Against the same
    tick with a flat completion payload; both on the trajectory path (the default) and on the general wave pipeline."""
    from zeebe_amd import workloads

    out, samples = {}, {}
    dup = b"\x82" + workloads.mp_str("step") + workloads.mp_int(1) + workloads.mp_str("step") + workloads.mp_int(2)
    flat = b"\x81" + workloads.mp_str("step") + workloads.mp_int(1)
    for wave_only in (False, True):
        for name, jp in (("flat", flat), ("exact", dup)):
            import copy

            b = copy.copy(a)
            b.wave_only = wave_only
            xml, pid, blob, offs, _, desc = workload("c1", n, 0)
            eng = make_engine("c1", n, b, 0, 1, 0)
            eng.deploy(xml, 100, 1)
            eng.set_job_payload(100, "t1", jp)
            eng.create_packed(pid, blob, offs)
            ms = []
            for it in range(steps + 1):
                eng.reset(keep_staged=True)
                t0 = time.perf_counter()
                st = eng.step()
                t1 = time.perf_counter()
                assert st["quiescent"] and st["merges"] == n, st
                if it:
                    ms.append((t1 - t0) * 1e3)
                print("exact-tree %s %s step %d: %.2f ms" % ("wave" if wave_only else "traj", name, it, (t1 - t0) * 1e3),
                      file=sys.stderr, flush=True)
            samples["%s_%s" % ("wave" if wave_only else "traj", name)] = _completion_sample(eng)
            eng.close()
            out["%s_%s" % ("wave" if wave_only else "traj", name)] = sum(ms) / len(ms)
    for p in ("traj", "wave"):
        out["%s_ratio" % p] = out["%s_exact" % p] / out["%s_flat" % p]
        # the results checked: the duplicate key keeps the first position and the last value (MsgPackDocumentIndexer),
        # so every exact-tree result is the structural merge's flat result with "step" 2 instead of 1
        flat, exact = samples["%s_flat" % p], samples["%s_exact" % p]
        assert len(exact) > 1000 and exact.keys() == flat.keys(), (p, len(exact), len(flat))
        for k, pairs in flat.items():
            assert exact[k] == [(a, 2 if a == "step" else b) for a, b in pairs], (p, k, exact[k], pairs)
        out["%s_checked" % p] = len(exact)
    out["workload"] = ("C1, %d instances per tick, every job completion payload with a duplicate key (the exact tree "
                       "for each of the %d default output merges) vs a flat completion payload; stepping ms per tick, "
                       "trajectory path and general wave pipeline" % (n, n))
    return out


def _completion_sample(eng, m=30000):
    """{workflow instance key: the process's final payload as (key, value) pairs} from the last m records of the tick
    (the last generations: every instance's END_EVENT / process ELEMENT_COMPLETED carries its merge result)."""
    import msgpack

    L = eng.log_size()
    out = {}
    for r in eng.records(L - m, m):
        v = msgpack.unpackb(r.value, raw=False)
        if r.record_type == 0 and v.get("activityId") == "chain" and r.intent == 9:  # the process's ELEMENT_COMPLETED
            out[v["workflowInstanceKey"]] = msgpack.unpackb(v["payload"], raw=False, object_pairs_hook=list)
    return out


def run_c5(a, rank, world, local_rank, dist):
    import socket

    import torch
    import torch.distributed as tdist

    import bench_extra

    if dist is None:  # the exchange driver needs a (one-rank) control plane
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(s.getsockname()[1]))
        s.close()
        tdist.init_process_group("gloo", rank=0, world_size=1)
        dist = tdist

    def barrier():
        dist.barrier()

    def reduce(v, op):
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t.item())

    bench_extra.run_c5(a, rank, world, local_rank, dist, barrier, lambda v: reduce(v, tdist.ReduceOp.MAX),
                       lambda v: reduce(v, tdist.ReduceOp.SUM))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
