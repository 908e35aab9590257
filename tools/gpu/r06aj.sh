set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06aj
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_messages.py -x -k "tokens or single_target or round_trip" -q --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { echo "msg tests failed"; tail -40 $O/pytest_msg.log; exit 1; }
tail -1 $O/pytest_msg.log
