#!/bin/bash
# Round-4 measurement set: the default bench line (C3 headline + extras + CPU baseline), kernel stats of the C3
# headline and of the C2 steady state, and PMC passes (HBM traffic) for the steady state, C3 wave-only and C4.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('C3', d['value']/1e9, 'G/s', d['ms_per_step'], 'ms', d['roofline']['kernel'], d['roofline']['frac']); [print(k, v['ms_per_step'], v['roofline']['frac']) for k, v in d.get('extras', {}).items()]"
timeout -k 10 300 python3 -u bench.py --config c1 --steps 20 --warmup 2 > $O/bench_c1.json 2> $O/bench_c1.err || { echo "c1 failed"; tail -5 $O/bench_c1.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -5 $O/bench_c5.err; exit 1; }
TAG=c3 BENCH_ARGS="--config c3" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c2s STEPS=5 BENCH_ARGS="--config c2 --steady" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c2w BENCH_ARGS="--config c2 --wave-only" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c5 BENCH_ARGS="--config c5" bash tools/gpu/prof_cfg.sh || exit 1
SQ="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
TAG=c2s_1000000 PMC_STEPS=3 BENCH_ARGS="--config c2 --steady --no-extras" PMC_SETS="FETCH_SIZE;WRITE_SIZE;$SQ" bash tools/gpu/run_gpu_pmc.sh || exit 1
PMC_SKIP_TICKS=1 python3 tools/pmc_summary.py gpurun_out/pmc_c2s_1000000 $O/pmc_c2s_1000000.json > $O/pmc_c2s_1000000.txt || exit 1
TAG=c3w_10000000 BENCH_ARGS="--config c3 --wave-only --no-extras" PMC_SETS="FETCH_SIZE;WRITE_SIZE;$SQ" bash tools/gpu/run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c3w_10000000 $O/pmc_c3w_10000000.json > $O/pmc_c3w_10000000.txt || exit 1
TAG=c2w_1000000 BENCH_ARGS="--config c2 --wave-only --no-extras" PMC_SETS="FETCH_SIZE;WRITE_SIZE;$SQ" bash tools/gpu/run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c2w_1000000 $O/pmc_c2w_1000000.json > $O/pmc_c2w_1000000.txt || exit 1
TAG=c3_10000000 BENCH_ARGS="--config c3 --no-extras" PMC_SETS="FETCH_SIZE;WRITE_SIZE;$SQ" bash tools/gpu/run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c3_10000000 $O/pmc_c3_10000000.json > $O/pmc_c3_10000000.txt || exit 1
TAG=c4_1000000 BENCH_ARGS="--config c4 --no-extras" PMC_SETS="FETCH_SIZE;WRITE_SIZE" bash tools/gpu/run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c4_1000000 $O/pmc_c4_1000000.json > $O/pmc_c4_1000000.txt || exit 1
head -12 $O/pmc_c2s_1000000.txt
