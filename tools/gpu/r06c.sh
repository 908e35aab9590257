set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r06c/suite.log 2>&1 && \
timeout -k 10 300 python -u tools/gpu/exact_line.py > gpurun_out/r06c/exact.json 2> gpurun_out/r06c/exact.err
