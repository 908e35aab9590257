set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ak
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/prof -o c3 --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo ok
