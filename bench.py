"""bench.py — BPMN element transitions/s on MI355X (BASELINE.json metric), one partition per GPU.

Workload (BASELINE.json configs[1]): a 20-service-task chain, 1,000,000 concurrent
instances per GPU (all CREATE commands injected before wave 0), job k completed by the canonical
harness with payload {"step": k}; every completion runs the default output merge. One "step" =
inject the staged 1M CREATE batch (already resident in HBM) and run every lockstep wave until the
partition is quiescent (~148 waves, ~169M records, 108M WORKFLOW_INSTANCE transitions).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process and one partition
per GPU, each with its own 1M instances (partitions never communicate for this workload:
weak scaling, no collective on the data path; the barrier + max-over-ranks timing use torch.distributed).

Prints ONE JSON line on rank 0 (contract in the task statement) with "roofline" and "cpu_baseline".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BYTES_PER_TRANSITION = 96  # 32 B row read + 32 B row write + 32 B record descriptor
DESC_BYTES = 32  # one zb_rec descriptor written per log record
# HBM bytes of the main emit kernel from the committed rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: separate
# runs of this script with --steps 1; tools/pmc_summary.py writes the file with the gfx950 correction)
PMC_FILE = os.path.join(ROOT, "profiles", "r01", "pmc_v7.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=("c2", "c3", "c5"), default="c2",
                    help="BASELINE.json configuration (default: C2, the headline metric); c3 / c5: bench_extra.py")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--instances", type=int, default=0, help="per GPU (default: C2/C5 1,000,000, C3 10,000,000)")
    ap.add_argument("--tasks", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=30_000, help="instances in the oracle CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--wave-only", action="store_true", help="force the general wave pipeline (no trajectory path)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on GPU 0 (multi-rank rehearsal on a one-GPU box; not a scaling run)")
    return ap.parse_args()


def cpu_baseline(n_inst, tasks):
    """The oracle (sequential C++ restatement, 1 thread) on a bounded sample of the same workload."""
    from oracle import zbref
    from zeebe_amd import bpmn, workloads

    xml = bpmn.chain_workflow(tasks).to_xml()
    o = zbref.Oracle()
    o.deploy(xml, 100, 1)
    for k in range(1, tasks + 1):
        o.set_job_payload(100, "t%d" % k, b"\x81" + workloads.mp_str("step") + workloads.mp_int(k))
    blob, offs = workloads.order_payloads(n_inst)
    for p in workloads.split(blob, offs):
        o.create("chain", p)
    n, secs = o.run_timed()
    transitions = (8 + 5 * tasks) * n_inst
    return {"value": transitions / secs, "unit": "transitions/s", "cores": 1, "kind": "port",
            "sample": "C2 chain of %d tasks, %d instances, %d records processed in %.2f s by oracle/zbref "
                      "(1 thread, sequential FIFO, canonical job harness)" % (tasks, n_inst, n, secs),
            "completed_instances_per_s": n_inst / secs}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        # Control plane only (barrier, max-over-ranks, sums): the C2 partitions never exchange data, so
        # there is no data-path collective (weak scaling). gloo keeps torch's own HIP runtime out of the
        # process: the engine (libzbgpu.so) drives its GPU through the system ROCm runtime and
        # synchronizes its own stream at the end of every zb_step.
        dist.init_process_group("gloo")

    if a.instances == 0:
        a.instances = 10_000_000 if a.config == "c3" else 1_000_000
    if a.config != "c2":
        return run_other(a, rank, world, local_rank, dist)

    from zeebe_amd import bpmn, workloads
    from zeebe_amd.engine import Engine

    n = a.instances
    recs_per_inst = 1 + (8 + 5 * a.tasks) + 3 * a.tasks  # CREATE + WF events + JOB CREATE/CREATED/COMPLETED
    eng = Engine(device=0 if a.same_device else local_rank, partition_id=rank, partition_count=world,
                 log_capacity=int(n * (recs_per_inst + 2)), row_capacity=int(n * (a.tasks + 2)),
                 arena_bytes=int(n * (48 + 48 * a.tasks)) + (64 << 20), wave_only=a.wave_only)
    xml = bpmn.chain_workflow(a.tasks).to_xml()
    eng.deploy(xml, 100, 1)
    for k in range(1, a.tasks + 1):
        eng.set_job_payload(100, "t%d" % k, b"\x81" + workloads.mp_str("step") + workloads.mp_int(k))
    # instance i of this partition: global instance id = rank * n + i (round-robin over partitions)
    blob, offs = workloads.order_payloads(n, start=rank * n)
    eng.create_packed("chain", blob, offs)

    def one_step():
        eng.reset(keep_staged=True)
        st = eng.step()
        assert st["quiescent"], st
        return st

    for _ in range(a.warmup):
        one_step()

    def barrier():
        if dist is not None:
            dist.barrier()  # every rank's zb_step has returned: its stream is drained

    barrier()
    t0 = time.perf_counter()
    tot = dict(main_ms=0.0, written=0, transitions=0, completed=0, kernel_ms=0.0, process_ms=0.0, emit_ms=0.0, aux_ms=0.0, launches=0, waves=0, merge_bytes=0, cond_bytes=0,
               records=0, path=0)
    for _ in range(a.steps):
        st = one_step()
        tot["transitions"] += st["transitions"]
        tot["completed"] += st["completed_instances"]
        tot["kernel_ms"] += st["wave_kernel_ms"]
        tot["main_ms"] += st["main_emit_kernel_ms"]
        tot["written"] += st["records_written"]
        tot["process_ms"] += st["process_kernel_ms"]
        tot["emit_ms"] += st["emit_kernel_ms"]
        tot["aux_ms"] += st["aux_kernel_ms"]
        tot["launches"] += st["launches"]
        tot["waves"] += st["waves"]
        tot["merge_bytes"] += st["merge_bytes"]
        tot["cond_bytes"] += st["condition_payload_bytes"]
        tot["records"] += st["records_processed"]
        tot["path"] = st["path"]
    barrier()
    elapsed = time.perf_counter() - t0

    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([tot["transitions"], tot["completed"]], dtype=torch.float64)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        all_transitions, all_completed = float(c[0]), float(c[1])
    else:
        all_transitions, all_completed = float(tot["transitions"]), float(tot["completed"])

    traffic, pmc_kernel = None, None
    if n == 1_000_000 and a.tasks == 20 and os.path.exists(PMC_FILE):
        with open(PMC_FILE) as f:
            pmc = json.load(f)
        traffic, pmc_kernel = pmc["main_traffic_bytes"], pmc["main_kernel"]

    if rank == 0:
        # path level (SURVEY §8d model): 96 B per transition + merge + condition bytes over every kernel of a step
        alg_bytes = BYTES_PER_TRANSITION * tot["transitions"] + tot["merge_bytes"] + tot["cond_bytes"]
        kernel_s = tot["kernel_ms"] / 1e3
        path_achieved = alg_bytes / kernel_s / 1e9 if kernel_s > 0 else 0.0
        # dominant kernel (the main emit launch, ~80% of device time): per launch it writes every record
        # descriptor of the batch and performs every output merge (reads job + scope documents, writes the
        # result) and condition evaluation; one launch per step
        main_bytes = DESC_BYTES * tot["written"] + tot["merge_bytes"] + tot["cond_bytes"]
        main_s = tot["main_ms"] / 1e3
        achieved = main_bytes / main_s / 1e9 if main_s > 0 else path_achieved
        out = {
            "metric": "BPMN element transitions/sec (+ completed instances/sec) per node; % HBM roofline",
            "value": all_transitions / elapsed,
            "unit": "transitions/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (SURVEY §8d C2: {\"orderId\": i} create payloads, {\"step\": k} job payloads)",
            "config": {"workload": "C2: 20-service-task chain, %d concurrent instances per GPU, canonical job "
                                   "harness, default output merges" % n,
                       "instances_per_gpu": n, "tasks": a.tasks, "partitions": world,
                       "parallelism": "partition-per-gpu"},
            "completed_instances_per_s": all_completed / elapsed,
            "records_processed_per_step_rank0": tot["records"] / a.steps,
            "wave_launches_per_step": tot["launches"] / a.steps,
            "kernel_ms_per_step": {"total": tot["kernel_ms"] / a.steps, "process_or_count": tot["process_ms"] / a.steps,
                                   "scan_emit": tot["emit_ms"] / a.steps, "aux": tot["aux_ms"] / a.steps},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "traffic_note": "HBM bytes per launch of %s (FETCH_SIZE x2 + WRITE_SIZE, separate "
                                         "rocprofv3 --pmc passes, profiles/r01/pmc_v7.json)" % pmc_kernel,
                         "kernel": {0: "zbg::k_emit (wave pipeline)", 1: "zbg::k_tmpl<false,false> (template emit)",
                                    2: "zbg::k_tmpl<true,false> (class-batch emit)"}.get(tot["path"], "?"),
                         "launches": a.steps, "avg_launch_us": tot["main_ms"] * 1e3 / a.steps,
                         "alg_bytes_per_launch": main_bytes / a.steps,
                         "alg_bytes_model": "32 B descriptor per record written + merge (job+scope+result) bytes "
                                            "+ condition payload bytes"},
            "path_roofline": {"achieved": path_achieved, "frac": path_achieved / HBM_PEAK_GBS, "unit": "GB/s",
                              "kernels": "every kernel of a step (count, scan, emit, commit)",
                              "kernel_launches": tot["launches"],
                              "alg_bytes_per_transition": BYTES_PER_TRANSITION, "alg_bytes_total": alg_bytes},
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.cpu_sample, a.tasks)
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def run_other(a, rank, world, local_rank, dist):
    import socket

    import torch
    import torch.distributed as tdist

    import bench_extra

    if dist is None and a.config == "c5":  # the exchange driver needs a (one-rank) control plane
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(s.getsockname()[1]))
        s.close()
        tdist.init_process_group("gloo", rank=0, world_size=1)
        dist = tdist

    def barrier():
        if dist is not None:
            dist.barrier()

    def reduce(v, op):
        if dist is None:
            return v
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t.item())

    fn = bench_extra.run_c3 if a.config == "c3" else bench_extra.run_c5
    fn(a, rank, world, local_rank, dist, barrier, lambda v: reduce(v, tdist.ReduceOp.MAX),
       lambda v: reduce(v, tdist.ReduceOp.SUM))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
