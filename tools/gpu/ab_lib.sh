#!/bin/bash
# A/B of whole product libraries on one box (box-to-box HBM rates differ by up to 1.8x: compare within a call).
# usage: LIBS="ab/libzbgpu_base.so ab/libzbgpu_new.so" [REPS=2] [BENCH_ARGS=...] bash tools/gpu/ab_lib.sh
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ab
mkdir -p $O
cp zeebe_amd/libzbgpu.so $O/.libzbgpu_head.so
for rep in $(seq ${REPS:-2}); do
  for l in $LIBS; do
    cp $l zeebe_amd/libzbgpu.so
    t=$(basename $l .so)
    ZB_AB_LIBRARY=1 timeout -k 10 300 python3 bench.py --no-extras --no-cpu-baseline --steps 5 ${BENCH_ARGS} > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; cp $O/.libzbgpu_head.so zeebe_amd/libzbgpu.so; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/$t.json').read().splitlines() if l.startswith('{')][-1]); b=d.get('step_breakdown_ms', {}); print('$t', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', {k: round(x,3) for k,x in b.items()})"
  done
done
cp $O/.libzbgpu_head.so zeebe_amd/libzbgpu.so
