#!/bin/bash
# PMC passes for the wave kernels (each counter group in its own rocprofv3 run, kernel trace only;
# never combined with -s/-r or API trace domains). Usage: PMC_SETS="FETCH_SIZE;WRITE_SIZE" ./run_gpu_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
INST=${INST:-1000000}
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
IFS=';' read -ra SETS <<< "${PMC_SETS:-FETCH_SIZE;WRITE_SIZE}"
i=0
for s in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $s --kernel-trace -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --instances $INST --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc/p$i.json 2> gpurun_out/pmc/p$i.err || { echo "pmc pass $i ($s) failed rc=$?"; tail -5 gpurun_out/pmc/p$i.err; exit 1; }
  echo "pass $i done: $s"
done
