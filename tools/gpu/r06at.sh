set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06at
mkdir -p $O
LIBS="ab/head.so ab/optin.so" REPS=2 OUT=$O/ab bash tools/gpu/wave_ab.sh || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_shared_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_shared.log 2>&1 || { tail -30 $O/pytest_shared.log; exit 1; }
tail -n 3 $O/pytest_shared.log
