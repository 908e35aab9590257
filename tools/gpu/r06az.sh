set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06az
mkdir -p $O
# k_pre over a wider grid (pre4 / pre16: 4x / 16x the wave grid) against the final library, C4 wave-only
LIBS="ab/final.so ab/pre4.so ab/pre16.so" REPS=2 CFGS=c4 OUT=$O/ab bash tools/gpu/wave_ab.sh || exit 1
LIBS="ab/final.so ab/pre4.so ab/pre16.so" CFG=c4 OUT=$O/prof bash tools/gpu/wave_prof.sh || exit 1
