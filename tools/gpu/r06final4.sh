set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06final4
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
ZB_CHECKED_LIBRARY=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_checked.log 2>&1 || { echo "checked suite failed"; tail -30 $O/pytest_gpu_checked.log; exit 1; }
tail -n 1 $O/pytest_gpu_checked.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -n 3 $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo ok
