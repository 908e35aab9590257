#!/bin/bash
# Round-5 PMC passes at HEAD (HBM traffic per launch / per tick + issue counters), installed into profiles/r05 of this
# tree so that the bench lines after them carry the traffic figures. Every pass under its own time limit; the first
# failure ends the script. usage: [CFGS="c3 c2w c2s c3w c4 c5"] bash tools/gpu/run_r05_pmc.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O profiles/r05
SQ="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
pmc() {  # tag, bench args, sets[, skip ticks]
  TAG=$1 BENCH_ARGS="$2" PMC_SETS="$3" PMC_STEPS=${PMC_STEPS:-1} bash tools/gpu/run_gpu_pmc.sh || return 1
  PMC_SKIP_TICKS=${4:-0} python3 tools/pmc_summary.py gpurun_out/pmc_$1 $O/pmc_$1.json > $O/pmc_$1.txt || return 1
  cp $O/pmc_$1.json $O/pmc_$1.txt profiles/r05/
}
for c in ${CFGS:-c3 c2w c2s c3w c4 c5}; do
  case $c in
    c3) pmc c3_10000000 "--config c3 --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1 ;;
    c2w) pmc c2w_1000000 "--config c2 --wave-only --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1 ;;
    c2s) PMC_STEPS=3 pmc c2s_1000000 "--config c2 --steady --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" 1 || exit 1 ;;
    c3w) pmc c3w_10000000 "--config c3 --wave-only --no-extras" "FETCH_SIZE;WRITE_SIZE" || exit 1 ;;
    c4) pmc c4_1000000 "--config c4 --no-extras" "FETCH_SIZE;WRITE_SIZE" || exit 1 ;;
    c5) pmc c5_1000000 "--config c5" "FETCH_SIZE;WRITE_SIZE" || exit 1 ;;
  esac
  echo "pmc $c done"
done
