#!/bin/bash
# Round-4 final measurement set at HEAD. PMC passes first (HBM traffic per launch / per tick), installed into
# profiles/r04 of this tree so that the bench lines after them carry the traffic figures; then the default bench
# line (C3 headline + extras + CPU baseline), C1 and C5 lines, and kernel statistics of C3, C2 steady, C2 wave-only
# and C5. Every GPU step under its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
SQ="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
pmc() {  # tag, bench args, sets[, skip ticks]
  TAG=$1 BENCH_ARGS="$2" PMC_SETS="$3" PMC_STEPS=${PMC_STEPS:-1} bash tools/gpu/run_gpu_pmc.sh || return 1
  PMC_SKIP_TICKS=${4:-0} python3 tools/pmc_summary.py gpurun_out/pmc_$1 $O/pmc_$1.json > $O/pmc_$1.txt || return 1
  cp $O/pmc_$1.json $O/pmc_$1.txt profiles/r04/
}
pmc c3_10000000 "--config c3 --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1
pmc c2w_1000000 "--config c2 --wave-only --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" || exit 1
PMC_STEPS=3 pmc c2s_1000000 "--config c2 --steady --no-extras" "FETCH_SIZE;WRITE_SIZE;$SQ" 1 || exit 1
pmc c3w_10000000 "--config c3 --wave-only --no-extras" "FETCH_SIZE;WRITE_SIZE" || exit 1
pmc c4_1000000 "--config c4 --no-extras" "FETCH_SIZE;WRITE_SIZE" || exit 1
pmc c5_1000000 "--config c5" "FETCH_SIZE;WRITE_SIZE" || exit 1
echo "pmc done"
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('C3', d['value']/1e9, 'G/s', d['ms_per_step'], 'ms', d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic']); [print(k, v['ms_per_step'], v['roofline']['frac'], v['roofline'].get('traffic')) for k, v in d.get('extras', {}).items()]"
timeout -k 10 300 python3 -u bench.py --config c1 --steps 20 --warmup 2 > $O/bench_c1.json 2> $O/bench_c1.err || { echo "c1 failed"; tail -5 $O/bench_c1.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -5 $O/bench_c5.err; exit 1; }
tail -1 $O/bench_c5.json | cut -c1-400
TAG=c3 BENCH_ARGS="--config c3" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c2s STEPS=5 BENCH_ARGS="--config c2 --steady" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c2w BENCH_ARGS="--config c2 --wave-only" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c5 BENCH_ARGS="--config c5" bash tools/gpu/prof_cfg.sh || exit 1
echo "final set done"
