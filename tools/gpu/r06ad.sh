set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ad
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_sys.json 2> $O/c5_sys.err || exit 1
timeout -k 10 300 python3 -u tools/gpu/rt_first.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_torch.json 2> $O/c5_torch.err || exit 1
timeout -k 10 300 python3 -u tools/gpu/exact_line.py > $O/exact.json 2> $O/exact.err || exit 1
echo ok
