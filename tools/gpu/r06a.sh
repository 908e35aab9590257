set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fast_frames.py tests/test_gpu_frames.py tests/test_gpu_parity.py > gpurun_out/r06a/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --jobs external --frames --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r06a/bench_frames.json 2> gpurun_out/r06a/bench_frames.err && \
timeout -k 10 300 python -u bench.py --jobs external --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r06a/bench_ext.json 2> gpurun_out/r06a/bench_ext.err
