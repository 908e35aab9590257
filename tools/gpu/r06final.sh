set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06final2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
ZB_CHECKED_LIBRARY=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_checked.log 2>&1 || { echo "checked suite failed"; tail -30 $O/pytest_gpu_checked.log; exit 1; }
tail -1 $O/pytest_gpu_checked.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
echo ok
