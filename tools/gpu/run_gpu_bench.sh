#!/bin/bash
# GPU bench + profile run (used with gpurun). Each GPU step has its own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-3}
INST=${INST:-1000000}
timeout -k 10 600 python bench.py --steps $STEPS --warmup 1 --instances $INST ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --instances $INST --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed rc=$?"; tail -20 gpurun_out/prof.err; exit 1; }
  find gpurun_out/prof -name '*stats*' | head
fi
