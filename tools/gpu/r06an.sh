set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06an
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fast_frames.py tests/test_gpu_frames.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "frames tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LIBS="ab/head.so ab/rot.so ab/head.so ab/rot.so" REPS=1 BENCH_ARGS="--frames --steps 8" timeout -k 10 800 bash tools/gpu/ab_lib.sh > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
