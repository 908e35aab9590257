set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06av
mkdir -p $O
# the capacity-overflow regressions first, alone (product, then guard-band build), then the rest
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_regressions.py -m gpu -x -v --timeout 120 --timeout-method thread -k overflow > $O/pytest_overflow.log 2>&1 || { tail -30 $O/pytest_overflow.log; exit 1; }
tail -n 2 $O/pytest_overflow.log
ZB_CHECKED_LIBRARY=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_regressions.py -m gpu -x -v --timeout 120 --timeout-method thread -k overflow > $O/pytest_overflow_checked.log 2>&1 || { tail -30 $O/pytest_overflow_checked.log; exit 1; }
tail -n 2 $O/pytest_overflow_checked.log
LIBS="ab/head.so ab/optin.so" REPS=1 OUT=$O/ab bash tools/gpu/wave_ab.sh || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
ZB_CHECKED_LIBRARY=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_checked.log 2>&1 || { echo "checked suite failed"; tail -30 $O/pytest_gpu_checked.log; exit 1; }
tail -n 1 $O/pytest_gpu_checked.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -n 3 $O/smoke.log
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29521 bench.py --config c4 --gpus 8 --same-device --instances 125000 --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/c4_8rank.json 2> $O/c4_8rank.err || { echo "c4 8-rank failed"; tail -20 $O/c4_8rank.err; exit 1; }
echo ok
