set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ax
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_shared_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_shared.log 2>&1 || { tail -40 $O/pytest_shared.log; exit 1; }
tail -n 6 $O/pytest_shared.log
