#!/bin/bash
# One rocprofv3 --pmc pass (issue counters, kernel trace only) of a bench configuration per library: the dynamic
# instruction counts of one kernel per measurement variant (tools/ab_variant.sh), summarised by tools/pmc_summary.py.
# usage: LIBS="ab/a.so ab/b.so" [KERNEL=k_tdrain_write] [BENCH_ARGS="--config c3"] [OUT=gpurun_out/pmc_ab] bash tools/gpu/pmc_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/pmc_ab}
mkdir -p $O
cp zeebe_amd/libzbgpu.so $O/.head.so
K=${KERNEL:-k_tdrain_write}
for l in $LIBS; do
  cp $l zeebe_amd/libzbgpu.so
  t=$(basename $l .so)
  ZB_AB_LIBRARY=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-trace -d $O/$t/p1 -o run --output-format csv -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:---config c3} > $O/$t.txt 2>&1 || { echo "$t failed"; tail -5 $O/$t.txt; cp $O/.head.so zeebe_amd/libzbgpu.so; exit 1; }
  python3 tools/pmc_summary.py $O/$t $O/$t.json > /dev/null 2>&1
  python3 - $O/$t.json $K $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, v in d.items():
    if sys.argv[2] in k:
        print("%-24s valu %6.1f M  salu %6.1f M  lds %6.1f M  smem %5.1f M  vmem_wr %5.1f M  cycles %5.2f M  valu_busy %.2f  wait %.2f" % (
            sys.argv[3], v["SQ_INSTS_VALU"] / 1e6, v["SQ_INSTS_SALU"] / 1e6, v["SQ_INSTS_LDS"] / 1e6, v["SQ_INSTS_SMEM"] / 1e6,
            v.get("SQ_INSTS_VMEM_WR", 0) / 1e6, v.get("kernel_cycles", 0) / 1e6, v.get("valu_busy", 0), v.get("wait_frac", 0)))
PY
done
cp $O/.head.so zeebe_amd/libzbgpu.so
