#!/bin/bash
# The exact-tree extras line (bench.run_exact_tree, C1 1M) for several whole libraries on one box.
# usage: LIBS="ab/a.so ab/b.so" [N=1000000] bash tools/gpu/exact_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/exact_ab
mkdir -p $O
cp zeebe_amd/libzbgpu.so $O/.head.so
for l in $LIBS; do
  cp $l zeebe_amd/libzbgpu.so
  t=$(basename $l .so)
  ZB_AB_LIBRARY=1 timeout -k 10 300 python3 -u -c "import sys; sys.argv=['bench.py']; import bench, json; a=bench.parse(); print(json.dumps(bench.run_exact_tree(a, n=${N:-1000000})))" > $O/$t.txt 2>&1 || { echo "$t failed"; tail -5 $O/$t.txt; cp $O/.head.so zeebe_amd/libzbgpu.so; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$t.txt').read().splitlines()[-1]); print('$t', {k: round(v, 3) for k, v in d.items() if k != 'workload'})"
done
cp $O/.head.so zeebe_amd/libzbgpu.so
