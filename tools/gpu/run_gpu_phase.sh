#!/bin/bash
# k_wave phase profile (ZB_PHASE_PROF=1): per-tile time in ticket / process / look-back / write.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
ZB_PHASE_PROF=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/phase.json 2> gpurun_out/phase.err || { echo "phase run failed rc=$?"; tail -20 gpurun_out/phase.err; exit 1; }
grep "zb phase" gpurun_out/phase.err | tail -2
cat gpurun_out/phase.json
