set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06p
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c5_$i.json 2> $O/bench_c5_$i.err || { echo "bench failed"; tail -5 $O/bench_c5_$i.err; exit 1; }; done
timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 6 > $O/c5_calls.txt 2>&1 || { echo "c5_calls failed"; tail -20 $O/c5_calls.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c5 --output-format csv -- python3 bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo ok
