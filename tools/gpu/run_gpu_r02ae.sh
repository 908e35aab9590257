#!/bin/bash
# PMC passes of the C3 default bench (no extras) with the fast drain: FETCH / WRITE, SQ sets; summary ->
# profiles/r02/pmc_c3_10000000.json (bench.py's roofline traffic); plus the final kernel trace + bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
S3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
S4="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
PMC_SETS="FETCH_SIZE;WRITE_SIZE;$S3;$S4" BENCH_ARGS="--no-extras" TAG=c3_10000000 ./run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c3_10000000 gpurun_out/pmc_c3_10000000.json | head -12
RUN_TAG=r02ae ./run_gpu_bench_prof.sh
