#!/bin/bash
# Round measurement set: GPU parity tests + smoke, the default bench line (extras + CPU baseline), then the
# kernel trace of the C3 headline command. Each GPU step has its own time limit; stop at the first failure.
# usage (repo root, on the GPU box): TAG=r03a bash tools/gpu/run_round.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  bash tools/gpu/run_tests.sh || exit 1
fi
timeout -k 10 600 python3 -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['step_breakdown_ms'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline'].get('path_frac')); print({k: (v['value']/1e9, v['ms_per_step']) for k, v in d.get('extras', {}).items()}); print(d.get('cpu_baseline', {}).get('value'), d.get('cpu_baseline', {}).get('multi_partition', {}).get('value'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -5 $O/prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
python3 - $O <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1] + '/kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
PY
