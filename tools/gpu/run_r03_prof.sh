#!/bin/bash
# C3 headline: PMC passes (one counter set per rocprofv3 run) + summary, then the C5 phase timing.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-c3} BENCH_ARGS="--no-extras ${BENCH_ARGS}" \
PMC_SETS="FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
  bash tools/gpu/run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG:-c3} gpurun_out/pmc_${TAG:-c3}.json > gpurun_out/pmc_${TAG:-c3}.txt 2>&1 || exit 1
