set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config c5 --steps 6 --warmup 1 --no-cpu-baseline > $O/b61.json 2> $O/b61.err || exit 1
timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/b102.json 2> $O/b102.err || exit 1
timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 1 --no-cpu-baseline > $O/b101.json 2> $O/b101.err || exit 1
timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 10 > $O/c5_calls.txt 2>&1 || exit 1
echo ok
