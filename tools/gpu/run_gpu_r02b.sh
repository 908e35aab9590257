#!/bin/bash
# round 2: new GPU tests, default bench (C3 10M + drain, extras, CPU baseline), kernel-trace profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conditions_product.py tests/test_gpu_extensions.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_b.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_b.log; exit 1; }
tail -3 gpurun_out/t_b.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > gpurun_out/prof_def.json 2> gpurun_out/prof_def.err || { echo "rocprof failed"; tail -20 gpurun_out/prof_def.err; exit 1; }
echo done
