#!/bin/bash
# Round-2 baseline: counters for the wave pipeline (C2 wave-only) and the template emit (C2 default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
S4="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2w -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --wave-only --no-cpu-baseline > gpurun_out/c2w.json 2> gpurun_out/c2w.err || { echo "c2w failed"; tail gpurun_out/c2w.err; exit 1; }
cat gpurun_out/c2w.json | head -c 600; echo
PMC_SETS="FETCH_SIZE;WRITE_SIZE;$S3;$S4" BENCH_ARGS="--wave-only" TAG=c2w ./run_gpu_pmc.sh || exit 1
PMC_SETS="$S3;$S4" BENCH_ARGS="" TAG=c2t ./run_gpu_pmc.sh || exit 1
echo done
