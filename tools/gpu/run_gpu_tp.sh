#!/bin/bash
# GPU tests, then the C3 bench line + kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
O=gpurun_out/${RUN_TAG:-tp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
RUN_TAG=${RUN_TAG:-tp} ./run_gpu_bench_prof.sh
