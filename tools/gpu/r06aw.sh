set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06aw
mkdir -p $O
# k_wave<false> / k_wave<true> (tmpl.so) against the runtime switch (optin.so) and the round-6 head (head.so)
LIBS="ab/head.so ab/optin.so ab/tmpl.so" REPS=2 CFGS=c2 OUT=$O/ab bash tools/gpu/wave_ab.sh || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_shared_gpu.py tests/test_gpu_regressions.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_shared.log 2>&1 || { tail -30 $O/pytest_shared.log; exit 1; }
tail -n 2 $O/pytest_shared.log
