set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/kab_pf LIBS="ab/head.so ab/kwave_pf.so ab/kwave_pfe.so ab/head.so ab/kwave_pf.so ab/kwave_pfe.so" BENCH_ARGS="--config c2 --wave-only" bash tools/gpu/kernel_ab.sh > gpurun_out/r06i_c2w.txt 2>&1 || exit 1
LIBS="ab/head.so ab/kwave_pf.so ab/kwave_pfe.so" REPS=2 BENCH_ARGS="--config c2 --steady --steps 12" bash tools/gpu/ab_lib.sh > gpurun_out/r06i_c2s.txt 2>&1 || exit 1
