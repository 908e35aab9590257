#!/bin/bash
# Round-5 final bench set at HEAD (after tools/gpu/run_r05_pmc.sh): the default bench line (C3 headline + extras + CPU
# baseline), the C1 and C5 lines, the steady line, and kernel statistics of C3, C2 steady, C2 wave-only and C5.
# Every GPU step under its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05
mkdir -p $O
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 800 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().splitlines()[-1]); print('C3', d['value']/1e9, 'G/s', d['ms_per_step'], 'ms', d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic']); [print(k, v.get('ms_per_step'), v.get('roofline', {}).get('frac'), v.get('roofline', {}).get('traffic')) for k, v in d.get('extras', {}).items() if isinstance(v, dict)]"
fi
if [ -z "$SKIP_LINES" ]; then
timeout -k 10 300 python3 -u bench.py --config c1 --steps 20 --warmup 2 > $O/bench_c1.json 2> $O/bench_c1.err || { echo "c1 failed"; tail -5 $O/bench_c1.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -5 $O/bench_c5.err; exit 1; }
tail -1 $O/bench_c5.json | cut -c1-300
timeout -k 10 400 python3 -u bench.py --config c2 --steady --steps 24 --warmup 1 > $O/bench_c2s.json 2> $O/bench_c2s.err || { echo "c2s failed"; tail -5 $O/bench_c2s.err; exit 1; }
tail -1 $O/bench_c2s.json | cut -c1-300
fi
if [ -z "$SKIP_PROF" ]; then
TAG=c3_r05 BENCH_ARGS="--config c3" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c2s_r05 STEPS=5 BENCH_ARGS="--config c2 --steady" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c2w_r05 BENCH_ARGS="--config c2 --wave-only" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c5_r05 BENCH_ARGS="--config c5" bash tools/gpu/prof_cfg.sh || exit 1
fi
echo "final set done"
