#!/bin/bash
# Kernel statistics of the wave pipeline (C2 wave-only stepping, tools/gpu/wave_exp.py) for several whole libraries on
# one box: rocprofv3 --kernel-trace --stats per library; prints the top kernels of each.
# usage: LIBS="ab/a.so ab/b.so" [CFG=c2] [OUT=gpurun_out/wave_prof] bash tools/gpu/wave_prof.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/wave_prof}
mkdir -p $O
cp zeebe_amd/libzbgpu.so $O/.head.so
for l in $LIBS; do
  cp $l zeebe_amd/libzbgpu.so
  t=$(basename $l .so)
  ZB_AB_LIBRARY=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run --output-format csv -- python3 -u tools/gpu/wave_exp.py ${CFG:-c2} 1000000 0 > $O/$t.txt 2>&1 || { echo "$t failed"; tail -5 $O/$t.txt; cp $O/.head.so zeebe_amd/libzbgpu.so; exit 1; }
  f=$(find $O/prof_$t -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats_$t.csv
  echo "== $t: $(grep stepping $O/$t.txt)"
  python3 - $O/kernel_stats_$t.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print("  %-50s %6s calls %9.1f us avg %8.2f ms total" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3,
                                                            float(r['TotalDurationNs']) / 1e6))
PY
done
cp $O/.head.so zeebe_amd/libzbgpu.so
