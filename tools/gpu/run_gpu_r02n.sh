#!/bin/bash
# job processor on the GPU: the new tests first, then the full GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02n
timeout -k 10 300 python -u -m pytest tests/test_gpu_jobs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02n/io.log 2>&1 || { echo "io tests failed"; tail -60 gpurun_out/r02n/io.log; exit 1; }
tail -1 gpurun_out/r02n/io.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02n/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r02n/tests.log; exit 1; }
tail -1 gpurun_out/r02n/tests.log
