#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_c.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_c.log; exit 1; }
tail -3 gpurun_out/t_c.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/bench_c.err; exit 1; }
cat gpurun_out/bench_c.json
