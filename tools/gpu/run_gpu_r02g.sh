#!/bin/bash
# drain write pass experiments (ZB_SER_EXP bits: 1 no encode, 2 no value stores, 4 no headers)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02g
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_messages.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02g/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r02g/tests.log; exit 1; }
tail -1 gpurun_out/r02g/tests.log
for x in 0 7; do
  ZB_SER_EXP=$x timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02g/x_$x.json 2> gpurun_out/r02g/x_$x.err || { echo "bench failed $x"; tail -5 gpurun_out/r02g/x_$x.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02g/x_$x.json'));print($x, round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
done
