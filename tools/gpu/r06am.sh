set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06am
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o ex --output-format csv -- python3 -u tools/gpu/exact_line.py > $O/exact.json 2> $O/exact.err || { tail -5 $O/exact.err; exit 1; }
echo ok
