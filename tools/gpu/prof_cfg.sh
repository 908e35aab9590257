#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of one bench configuration; top kernels by total time.
# usage: TAG=c2w BENCH_ARGS="--config c2 --wave-only" bash tools/gpu/prof_cfg.sh
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/prof_${TAG:-x}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > $O/bench.json 2> $O/prof.err || { echo "prof failed"; tail -5 $O/prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats.csv
python3 - $O <<'PY'
import csv, json, sys
d = json.loads([l for l in open(sys.argv[1] + '/bench.json').read().splitlines() if l.startswith('{')][-1])
print(round(d['value'] / 1e9, 3), 'G/s', round(d['ms_per_step'], 3), 'ms/step', {k: round(x, 3) for k, x in d.get('step_breakdown_ms', {}).items()})
rows = list(csv.DictReader(open(sys.argv[1] + '/kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('%-70s %6s calls %9.1f us avg %6.1f%%' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e3, 100 * float(r['TotalDurationNs']) / tot))
PY
