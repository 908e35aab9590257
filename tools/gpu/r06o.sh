set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 6 > $O/c5_calls.txt 2>&1 || { echo "c5_calls failed"; tail -20 $O/c5_calls.txt; exit 1; }
for i in 1 2; do timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_$i.json 2> $O/bench_c5_$i.err || { echo "bench failed"; tail -5 $O/bench_c5_$i.err; exit 1; }; done
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-extras --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench c3 failed"; tail -5 $O/bench_c3.err; exit 1; }
echo ok
