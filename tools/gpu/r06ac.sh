set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ac
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_messages.py tests/test_gpu_regressions.py tests/test_gpu_races.py -x -q --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { echo "msg tests failed"; tail -30 $O/pytest_msg.log; exit 1; }
tail -1 $O/pytest_msg.log
timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_sys.json 2> $O/c5_sys.err || exit 1
timeout -k 10 300 python3 -u tools/gpu/rt_first.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_torch.json 2> $O/c5_torch.err || exit 1
LIBS="ab/head.so ab/xl128k.so ab/xl128k_16.so ab/xl256k_16.so ab/xl128k.so ab/head.so" timeout -k 10 900 bash tools/gpu/exact_ab.sh > $O/exact_ab.txt 2>&1 || { tail -5 $O/exact_ab.txt; exit 1; }
echo ok
