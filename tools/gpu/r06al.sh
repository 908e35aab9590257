set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06al
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-extras --no-cpu-baseline > $O/c3_$i.json 2> $O/c3_$i.err || exit 1; done
echo ok
