set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fast_frames.py tests/test_gpu_frames.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
OUT=gpurun_out/kab_c3f LIBS="ab/head.so ab/frames128.so ab/head.so ab/frames128.so" BENCH_ARGS="--config c3 --frames" bash tools/gpu/kernel_ab.sh > $O/ab.txt 2>&1 || exit 1
echo done
