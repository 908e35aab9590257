#!/bin/bash
# Same-box A/B of whole product libraries on the wave pipeline (tools/gpu/wave_exp.py): every library in LIBS runs
# C2 and C4 wave-only stepping, REPS times, back to back; then the phase split of the current tree's phases build.
# usage (from the repo root, on the GPU box): LIBS="ab/a.so ab/b.so" [REPS=2] [OUT=gpurun_out/wave_ab] bash tools/gpu/wave_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=${OUT:-gpurun_out/wave_ab}
mkdir -p $O
cp zeebe_amd/libzbgpu.so $O/.head.so
for rep in $(seq ${REPS:-2}); do
  for l in $LIBS; do
    cp $l zeebe_amd/libzbgpu.so
    t=$(basename $l .so)
    for cfg in ${CFGS:-c2 c4}; do
      ZB_AB_LIBRARY=1 timeout -k 10 200 python3 -u tools/gpu/wave_exp.py $cfg 1000000 0 > $O/$t.$cfg.$rep.txt 2>&1 || { echo "$t $cfg failed"; tail -5 $O/$t.$cfg.$rep.txt; cp $O/.head.so zeebe_amd/libzbgpu.so; exit 1; }
      echo "$t: $(cat $O/$t.$cfg.$rep.txt | tail -1)"
    done
  done
done
cp $O/.head.so zeebe_amd/libzbgpu.so
if [ -n "$PHASES" ]; then
  timeout -k 10 200 python3 -u tools/gpu/phases.py c2 > $O/phases_c2.txt 2>&1 || { tail -5 $O/phases_c2.txt; exit 1; }
  tail -2 $O/phases_c2.txt
fi
