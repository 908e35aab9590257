#!/bin/bash
# Per-kernel device time of one bench configuration for several whole libraries on one box (measurement variants
# built by tools/ab_variant.sh): rocprofv3 --kernel-trace --stats per library, the top kernels of each.
# usage: LIBS="ab/a.so ab/b.so" [BENCH_ARGS="--config c3"] [OUT=gpurun_out/kernel_ab] bash tools/gpu/kernel_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/kernel_ab}
mkdir -p $O
cp zeebe_amd/libzbgpu.so $O/.head.so
for l in $LIBS; do
  cp $l zeebe_amd/libzbgpu.so
  t=$(basename $l .so)
  ZB_AB_LIBRARY=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run --output-format csv -- python3 -u bench.py --no-extras --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; cp $O/.head.so zeebe_amd/libzbgpu.so; exit 1; }
  f=$(find $O/prof_$t -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats_$t.csv
  echo "== $t"
  python3 - $O/kernel_stats_$t.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:7]:
    print("  %-50s %6s calls %9.1f us avg" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
cp $O/.head.so zeebe_amd/libzbgpu.so
