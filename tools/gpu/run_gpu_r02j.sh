#!/bin/bash
# k_wave profile: kernel trace + counters on C2 wave-only (tag c2w_1000000)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02j
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02j/prof_c2w -o run --output-format csv -- python3 bench.py --config c2 --wave-only --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02j/c2w.json 2> gpurun_out/r02j/c2w.err || { echo "c2w failed"; tail -5 gpurun_out/r02j/c2w.err; exit 1; }
S3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
S4="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
PMC_SETS="FETCH_SIZE;WRITE_SIZE;$S3;$S4" BENCH_ARGS="--config c2 --wave-only --no-extras" TAG=c2w_1000000 ./run_gpu_pmc.sh || exit 1
echo done
