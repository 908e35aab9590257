set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ae
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_exact_scale.py tests/test_gpu_payload_shapes.py tests/test_gpu_iomapping.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exact.log 2>&1 || { echo "exact tests failed"; tail -30 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
timeout -k 10 300 python3 -u tools/gpu/exact_line.py > $O/exact.json 2> $O/exact.err || exit 1
timeout -k 10 300 python3 -u tools/gpu/exact_line.py > $O/exact2.json 2> $O/exact2.err || exit 1
echo ok
