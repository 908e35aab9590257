set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ba
mkdir -p $O
# k_pre staging the chunk's records through LDS (prelds.so) against the final library: C4 wave-only + k_pre statistics
LIBS="ab/final.so ab/prelds.so" REPS=2 CFGS=c4 OUT=$O/ab bash tools/gpu/wave_ab.sh || exit 1
LIBS="ab/final.so ab/prelds.so" CFG=c4 OUT=$O/prof bash tools/gpu/wave_prof.sh || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c4 or parallel or cancel or fork or join or scope or regression or shared or wave" > $O/pytest_sel.log 2>&1 || { tail -30 $O/pytest_sel.log; exit 1; }
tail -n 1 $O/pytest_sel.log
