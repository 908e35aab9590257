#!/bin/bash
# wave-grid experiment: C2 wave-only stepping (no drain), sized grid vs fixed grids, kernel stats per variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
mkdir -p gpurun_out/grid
for g in 0 4096 1024; do
  ZB_WAVE_GRID=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/grid/g$g -o run -- python3 -u bench.py --config c2 --wave-only --no-drain --no-extras --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/grid/b$g.json 2> gpurun_out/grid/b$g.err || { echo "failed g=$g"; tail -5 gpurun_out/grid/b$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/grid/b$g.json'));print($g, d['value']/1e9, d['ms_per_step'], d['step_breakdown_ms'])"
done
