set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/kab_c2w LIBS="ab/head.so ab/kwave_w3.so" BENCH_ARGS="--config c2 --wave-only" bash tools/gpu/kernel_ab.sh > gpurun_out/r06e_c2w.txt 2>&1 || exit 1
OUT=gpurun_out/kab_c3 LIBS="ab/head.so ab/tdrain_lane.so" BENCH_ARGS="--config c3" bash tools/gpu/kernel_ab.sh > gpurun_out/r06e_c3.txt 2>&1 || exit 1
LIBS="ab/head.so ab/kwave_w3.so ab/head.so ab/kwave_w3.so" REPS=1 BENCH_ARGS="--config c2 --steady --steps 12" bash tools/gpu/ab_lib.sh > gpurun_out/r06e_c2s.txt 2>&1 || exit 1
