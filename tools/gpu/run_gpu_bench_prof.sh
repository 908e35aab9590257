#!/bin/bash
# C3 bench line + kernel trace of the same command (no tests)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-bp}
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-extras --no-cpu-baseline ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['step_breakdown_ms'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['achieved'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS} > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -5 $O/prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
python3 - $O <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1] + '/kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
PY
