set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 3 > $O/c5_calls.txt 2>&1 || { echo "c5_calls failed"; tail -20 $O/c5_calls.txt; exit 1; }
timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench failed"; tail -5 $O/bench_c5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c5 -- python3 bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_c5.csv \;
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace_c5.csv \;
echo ok
