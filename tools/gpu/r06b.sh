set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r06b/suite.log 2>&1
