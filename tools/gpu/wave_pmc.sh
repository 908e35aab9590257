#!/bin/bash
# HBM traffic of the wave pipeline's kernels (C2 wave-only stepping, tools/gpu/wave_exp.py) for several whole
# libraries on one box: two rocprofv3 --pmc passes per library (FETCH_SIZE, WRITE_SIZE; kernel trace only), summarised
# per kernel by tools/pmc_summary.py.
# usage: LIBS="ab/a.so ab/b.so" [CFG=c2] [OUT=gpurun_out/wave_pmc] bash tools/gpu/wave_pmc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/wave_pmc}
mkdir -p $O
cp zeebe_amd/libzbgpu.so $O/.head.so
for l in $LIBS; do
  cp $l zeebe_amd/libzbgpu.so
  t=$(basename $l .so)
  i=0
  mkdir -p $O/pmc_$t
  for s in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    ZB_AB_LIBRARY=1 timeout -s KILL 150 rocprofv3 --pmc $s --kernel-trace -d $O/pmc_$t/p$i -o run --output-format csv -- python3 -u tools/gpu/wave_exp.py ${CFG:-c2} 1000000 0 > $O/pmc_$t/p$i.txt 2>&1 || { echo "$t pass $s failed"; tail -5 $O/pmc_$t/p$i.txt; cp $O/.head.so zeebe_amd/libzbgpu.so; exit 1; }
    echo "$s" > $O/pmc_$t/p$i.set
  done
  python3 tools/pmc_summary.py $O/pmc_$t $O/pmc_$t.json > $O/pmc_$t.txt 2>&1 || true
  echo "== $t"
  python3 - $O/pmc_$t.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = d.get("kernels", d)
for k, v in sorted(ks.items(), key=lambda kv: -float(kv[1].get("hbm_bytes", 0) or 0) * kv[1].get("dispatches", 1))[:6]:
    n = v.get("dispatches", 1)
    print("  %-40s %5d dispatches  hbm total %8.1f MB  (fetch %8.1f MB x2, write %8.1f MB)" % (
        k[:40], n, float(v.get("hbm_bytes", 0) or 0) * n / 2**20, float(v.get("FETCH_SIZE", 0) or 0) * n / 1024,
        float(v.get("WRITE_SIZE", 0) or 0) * n / 1024))
PY
done
cp $O/.head.so zeebe_amd/libzbgpu.so
