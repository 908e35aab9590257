#!/bin/bash
# PMC passes over one bench.py run each (kernel trace only; never combined with -s/-r or API trace
# domains). Each pass is its own rocprofv3 run with at most one counter group per hardware block budget.
# Usage: PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES" BENCH_ARGS="--wave-only" TAG=c2w ./run_gpu_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
TAG=${TAG:-run}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${PMC_SETS:-FETCH_SIZE;WRITE_SIZE}"
i=0
for s in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $s --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps ${PMC_STEPS:-1} --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pmc pass $i ($s) failed rc=$?"; tail -5 $OUT/p$i.err; exit 1; }
  echo "$s" > $OUT/p$i.set
  echo "pass $i done: $s"
done
