#!/bin/bash
# Issue / LDS counters of one kernel on a bench configuration (one rocprofv3 --pmc pass per counter set, kernel trace
# only), averaged over that kernel's dispatches by tools/pmc_summary.py.
# usage: [KERNEL=k_tdrain_write] [BENCH_ARGS="--config c3"] [OUT=gpurun_out/lds_pmc] bash tools/gpu/lds_pmc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/lds_pmc}
mkdir -p $O
K=${KERNEL:-k_tdrain_write}
i=0
for s in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  ZB_AB_LIBRARY=1 timeout -s KILL 200 rocprofv3 --pmc $s --kernel-trace -d $O/p$i -o run --output-format csv -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:---config c3} > $O/p$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.txt; exit 1; }
done
python3 tools/pmc_summary.py $O $O/summary.json > $O/summary.log 2>&1 || { tail -5 $O/summary.log; exit 1; }
python3 - $O/summary.json $K <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.get("kernels", d).items():
    if sys.argv[2] in k:
        print(k)
        for c, x in sorted(v.items()):
            print("  %-28s %s" % (c, x))
PY
