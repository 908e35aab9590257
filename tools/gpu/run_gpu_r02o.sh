#!/bin/bash
# drain write pass: plain vs non-temporal output stores (C3 10M default bench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02o
for nt in 0 1; do
  ZB_SER_NT=$nt timeout -k 10 300 python3 -u bench.py --no-extras --no-cpu-baseline --steps 5 > gpurun_out/r02o/c3_nt$nt.json 2> gpurun_out/r02o/c3_nt$nt.err || { echo "c3 nt=$nt failed"; tail -5 gpurun_out/r02o/c3_nt$nt.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r02o/c3_nt$nt.json'));print('nt=$nt', round(d['value']/1e9,3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['step_breakdown_ms'].items()})"
done
