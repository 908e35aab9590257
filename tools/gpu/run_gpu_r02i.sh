#!/bin/bash
# fused wave kernel (k_wave): full GPU suite, then C2 wave-only / C4 fused vs three-kernel pipeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02i/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r02i/tests.log | head -20; tail -30 gpurun_out/r02i/tests.log; exit 1; }
tail -2 gpurun_out/r02i/tests.log
for fz in 1 0; do
  ZB_WAVE_FUSED=$fz timeout -k 10 300 python3 -u bench.py --config c2 --wave-only --no-drain --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02i/c2w_$fz.json 2> gpurun_out/r02i/c2w_$fz.err || { echo "c2w failed $fz"; tail -5 gpurun_out/r02i/c2w_$fz.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02i/c2w_$fz.json'));print('c2w fused=$fz', round(d['value']/1e9,3), round(d['ms_per_step'],3))"
  ZB_WAVE_FUSED=$fz timeout -k 10 300 python3 -u bench.py --config c4 --no-drain --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02i/c4_$fz.json 2> gpurun_out/r02i/c4_$fz.err || { echo "c4 failed $fz"; tail -5 gpurun_out/r02i/c4_$fz.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02i/c4_$fz.json'));print('c4 fused=$fz', round(d['value']/1e9,3), round(d['ms_per_step'],3))"
done
