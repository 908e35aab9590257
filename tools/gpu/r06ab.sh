set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ab
mkdir -p $O
LIBS="ab/head.so ab/xl128k.so ab/xl128k_16.so ab/xl256k_16.so ab/xl128k.so ab/head.so" timeout -k 10 900 bash tools/gpu/exact_ab.sh > $O/exact_ab.txt 2>&1 || { tail -5 $O/exact_ab.txt; exit 1; }
echo ok
