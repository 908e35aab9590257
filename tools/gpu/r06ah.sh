set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ah
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --config c5 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --config c1 > $O/c1.json 2> $O/c1.err || { tail -5 $O/c1.err; exit 1; }
echo ok
