#!/bin/bash
# Serializer counters on the default bench (C3 10M): two-pass with value templates (tag c3_10000000) and with
# the generic encoder (tag c3g), plus the kernel-trace summary of the default command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
S4="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/c3.json 2> gpurun_out/c3.err || { echo "c3 failed"; tail gpurun_out/c3.err; exit 1; }
head -c 400 gpurun_out/c3.json; echo
PMC_SETS="FETCH_SIZE;WRITE_SIZE;$S3;$S4" BENCH_ARGS="--no-extras" TAG=c3_10000000 ./run_gpu_pmc.sh || exit 1
ZB_SER_TMPL=0 PMC_SETS="FETCH_SIZE;WRITE_SIZE;$S3;$S4" BENCH_ARGS="--no-extras" TAG=c3g ./run_gpu_pmc.sh || exit 1
echo done
