#!/bin/bash
# log frames: full GPU parity suite (every compare also checks frames), C3 default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02l/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r02l/tests.log; exit 1; }
tail -1 gpurun_out/r02l/tests.log
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02l/c3.json 2> gpurun_out/r02l/c3.err || { echo "c3 failed"; tail -5 gpurun_out/r02l/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r02l/c3.json'));print('c3', round(d['value']/1e9,3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
