#!/bin/bash
# GPU parity tests + C3 bench + kernel trace (drain: tile-offset scan, LDS fast encoder, multi-workgroup payload sum)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
O=gpurun_out/${RUN_TAG:-r02u}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 bench.py --no-extras --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['step_breakdown_ms'], d['roofline']['frac'], d['roofline']['achieved'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/c3_prof.json 2> $O/c3_prof.err || { echo "prof failed"; tail -5 $O/c3_prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
python3 - $O <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1] + '/kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
PY
