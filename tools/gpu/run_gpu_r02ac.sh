#!/bin/bash
# GPU tests, then same-box A/B of the class emit (instance order vs class-uniform)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
O=gpurun_out/${RUN_TAG:-r02ac}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
RUN_TAG=${RUN_TAG:-r02ac} AB_VARS="ZB_TMPL_IO=1;ZB_TMPL_IO=0" ./run_gpu_ab.sh
