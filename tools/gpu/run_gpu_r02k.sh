#!/bin/bash
# windowed drain write pass: GPU parity subset, C3 default bench, C2 wave-only with drain
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02k/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r02k/tests.log; exit 1; }
tail -1 gpurun_out/r02k/tests.log
timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02k/c3.json 2> gpurun_out/r02k/c3.err || { echo "c3 failed"; tail -5 gpurun_out/r02k/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r02k/c3.json'));print('c3', round(d['value']/1e9,3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
timeout -k 10 300 python3 -u bench.py --config c2 --wave-only --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02k/c2w.json 2> gpurun_out/r02k/c2w.err || { echo "c2w failed"; tail -5 gpurun_out/r02k/c2w.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r02k/c2w.json'));print('c2w', round(d['value']/1e9,3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
