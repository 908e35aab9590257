#!/bin/bash
# Round-6 measurement set: PMC passes (HBM traffic per launch + issue counters) of the C3 headline (integration job mode,
# values + headers) and of the C3 log-frame line, installed into profiles/r06; then the default bench line (which reads
# them), and kernel statistics of both C3 lines. Every GPU step under its own time limit; the first failure ends it.
# usage: [SKIP_PMC=1] [SKIP_BENCH=1] [SKIP_PROF=1] [R=r06x] bash tools/gpu/run_r06_prof.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=${R:-r06}
O=gpurun_out/$R
mkdir -p $O profiles/r06
SQ="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
pmc() {  # tag, bench args, sets
  TAG=$1 BENCH_ARGS="$2" PMC_SETS="$3" PMC_STEPS=${PMC_STEPS:-1} bash tools/gpu/run_gpu_pmc.sh || return 1
  python3 tools/pmc_summary.py gpurun_out/pmc_$1 $O/pmc_$1.json > $O/pmc_$1.txt || return 1
  cp $O/pmc_$1.json $O/pmc_$1.txt profiles/r06/
}
if [ -z "$SKIP_PMC" ]; then
  for c in ${CFGS:-c3 c3f}; do
    case $c in
      c3) pmc c3_10000000 "--config c3 --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1 ;;
      c3f) pmc c3f_10000000 "--config c3 --frames --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1 ;;
      c2w) pmc c2w_1000000 "--config c2 --wave-only --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1 ;;
      c2s) PMC_STEPS=3 pmc c2s_1000000 "--config c2 --steady --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1 ;;
      c5) pmc c5_1000000 "--config c5" "FETCH_SIZE;WRITE_SIZE" || exit 1 ;;
    esac
    echo "pmc $c done"
  done
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 800 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -5 $O/bench_default.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().splitlines()[-1]); print('C3', d['value']/1e9, 'G/s', d['ms_per_step'], 'ms', d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic']); [print(k, v.get('ms_per_step'), v.get('roofline', {}).get('frac'), v.get('roofline', {}).get('traffic')) for k, v in d.get('extras', {}).items() if isinstance(v, dict)]"
fi
if [ -z "$SKIP_PROF" ]; then
  TAG=c3_$R BENCH_ARGS="--config c3" bash tools/gpu/prof_cfg.sh || exit 1
  TAG=c3f_$R BENCH_ARGS="--config c3 --frames" bash tools/gpu/prof_cfg.sh || exit 1
  cp gpurun_out/prof_c3_$R/kernel_stats.csv profiles/r06/kernel_stats_c3_$R.csv
  cp gpurun_out/prof_c3f_$R/kernel_stats.csv profiles/r06/kernel_stats_c3f_$R.csv
fi
echo "r06 set done"
