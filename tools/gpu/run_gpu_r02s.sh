#!/bin/bash
# kernel trace of the C3 default bench (per-kernel averages)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02s/prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r02s/c3.json 2> gpurun_out/r02s/c3.err || { echo "prof failed"; tail -5 gpurun_out/r02s/c3.err; exit 1; }
f=$(find gpurun_out/r02s/prof -name '*kernel_stats.csv' | head -1); cp $f gpurun_out/r02s/kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r02s/kernel_stats.csv')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms total')
PY
