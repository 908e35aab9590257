#!/bin/bash
# Round-5 bisection of the C2 wave-only regression (r03 -> r04 -> HEAD): stepping time of every library in LIBS on one
# box (tools/gpu/wave_ab.sh, C2 only, one repetition), then the HBM traffic of the wave kernels for PMC_LIBS
# (tools/gpu/wave_pmc.sh), then the exact-tree line at a reduced size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=${OUT:-gpurun_out/r05_bisect}
mkdir -p $O
OUT=$O/ab REPS=1 CFGS=c2 bash tools/gpu/wave_ab.sh || exit 1
if [ -n "$PMC_LIBS" ]; then
  LIBS="$PMC_LIBS" OUT=$O/pmc bash tools/gpu/wave_pmc.sh || exit 1
fi
if [ -n "$EXACT_N" ]; then
  timeout -k 10 300 python3 -u -c "
import json, sys, bench
sys.argv = ['bench.py', '--steps', '1']
a = bench.parse()
print(json.dumps(bench.run_exact_tree(a, n=$EXACT_N, steps=2)))
" > $O/exact_tree.txt 2>&1 || { tail -20 $O/exact_tree.txt; exit 1; }
  tail -1 $O/exact_tree.txt
fi
