set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ap
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_classes.py tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_fast_frames.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-extras --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
for i in 1 2; do timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-extras --no-cpu-baseline > $O/c3_$i.json 2> $O/c3_$i.err || exit 1; done
echo ok
