#!/bin/bash
# persistent drain write pass: parity tests that drain, then C3 10M bench with grid sweep (3 / 2 / 4 per CU, and one per tile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_properties.py tests/test_gpu_extensions.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02f/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r02f/tests.log; exit 1; }
tail -1 gpurun_out/r02f/tests.log
for g in 768 512 1024 100000000; do
  ZB_SER_GRID=$g timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02f/ser_$g.json 2> gpurun_out/r02f/ser_$g.err || { echo "bench failed $g"; tail -5 gpurun_out/r02f/ser_$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02f/ser_$g.json'));print($g, round(d['value']/1e9,3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
done
