#!/bin/bash
# serializer two-pass vs single-pass after the per-workgroup partial fix; C2 wave-only after the k_merge/k_cond stats fix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02h
for mode in two fused; do
  ZB_SER_MODE=$mode timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02h/$mode.json 2> gpurun_out/r02h/$mode.err || { echo "bench failed $mode"; tail -5 gpurun_out/r02h/$mode.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02h/$mode.json'));print('$mode', round(d['value']/1e9,3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02h/prof_c2w -o run --output-format csv -- python3 bench.py --config c2 --wave-only --no-drain --no-extras --no-cpu-baseline --steps 3 > gpurun_out/r02h/c2w.json 2> gpurun_out/r02h/c2w.err || { echo "c2w failed"; tail -5 gpurun_out/r02h/c2w.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r02h/c2w.json'));print('c2w', round(d['value']/1e9,3), round(d['ms_per_step'],3))"
