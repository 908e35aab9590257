#!/bin/bash
# Round-2 measurement set at HEAD: PMC passes of the C3 default bench (FETCH / WRITE + two SQ sets) ->
# profiles/r02/pmc_c3_10000000.json, then the full default bench line (extras + CPU baseline) and the kernel
# trace of the default command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
S3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
S4="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_LEVEL_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
PMC_SETS="FETCH_SIZE;WRITE_SIZE;$S3;$S4" BENCH_ARGS="--no-extras" TAG=c3_10000000 ./run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c3_10000000 gpurun_out/pmc_c3_10000000.json | head -4
cp gpurun_out/pmc_c3_10000000.json profiles/r02/pmc_c3_10000000.json
O=gpurun_out/${RUN_TAG:-r02ag}
mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench_full.json 2> $O/bench_full.err || { echo "full bench failed"; tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_full.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic']); print({k: (v['value'] / 1e9, v['ms_per_step']) for k, v in d.get('extras', {}).items()}); print(d['cpu_baseline']['value'], d['cpu_baseline']['multi_partition']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -5 $O/prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
head -4 $O/kernel_stats.csv | cut -c1-150
