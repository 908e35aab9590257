set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_exact_scale.py tests/test_gpu_payload_shapes.py tests/test_gpu_iomapping.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -5 $O/tests.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u tools/gpu/exact_line.py > $O/exact.json 2> $O/exact.err || { echo "prof failed"; tail -5 $O/exact.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/kernel_stats_exact.csv
echo done
