set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ay
mkdir -p $O
# what the per-wave k_merge_gen launch costs (nomg.so: not launched; valid for C2's flat payloads only) + the final
# library's C2 / C4 wave-only kernel statistics
LIBS="ab/final.so ab/nomg.so" REPS=2 CFGS=c2 OUT=$O/ab bash tools/gpu/wave_ab.sh || exit 1
LIBS="ab/final.so" CFG=c2 OUT=$O/prof_c2 bash tools/gpu/wave_prof.sh || exit 1
LIBS="ab/final.so" CFG=c4 OUT=$O/prof_c4 bash tools/gpu/wave_prof.sh || exit 1
