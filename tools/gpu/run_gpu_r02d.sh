#!/bin/bash
# GPU suite, then serializer A/B (two-pass vs single-pass, templates on/off) on C3 10M and the wave grid sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02d/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r02d/tests.log; exit 1; }
tail -2 gpurun_out/r02d/tests.log
for mode in two fused; do for t in 1 0; do
  ZB_SER_MODE=$mode ZB_SER_TMPL=$t timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02d/ser_${mode}_$t.json 2> gpurun_out/r02d/ser_${mode}_$t.err || { echo "bench failed $mode $t"; tail -5 gpurun_out/r02d/ser_${mode}_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02d/ser_${mode}_$t.json'));print('$mode', $t, round(d['value']/1e9,3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
done; done
for g in 0 512 1024 2048; do
  ZB_WAVE_GRID=$g timeout -k 10 300 python3 -u bench.py --config c2 --wave-only --no-drain --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02d/c2w_$g.json 2> gpurun_out/r02d/c2w_$g.err || { echo "c2w failed $g"; tail -5 gpurun_out/r02d/c2w_$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02d/c2w_$g.json'));print('c2w', $g, round(d['value']/1e9,3), round(d['ms_per_step'],3))"
done
