#!/bin/bash
# Round-3 measurement set, part 1: the C3 headline PMC passes (profiles/r03/pmc_c3_10000000.json feeds bench.py's
# roofline traffic), then the C1 (BASELINE configs[0], 10k) and C5 bench lines with their CPU baselines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
TAG=c3_10000000 bash tools/gpu/run_r03_prof.sh || exit 1
timeout -k 10 300 python3 -u bench.py --config c1 --steps 20 --warmup 2 > $O/bench_c1.json 2> $O/bench_c1.err || { echo "c1 failed"; tail -5 $O/bench_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c1.json')); print('C1', d['value']/1e6, 'M/s', d['ms_per_step'], 'ms', d['cpu_baseline']['value']/1e6, d['cpu_baseline']['multi_partition']['value']/1e6)"
timeout -k 10 300 python3 -u bench.py --config c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -5 $O/bench_c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); print('C5', d['value']/1e9, 'G/s', d['ms_per_step'], 'ms')"
