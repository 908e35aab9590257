set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/sys -o c5 --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/sys.log 2>&1 || { tail -5 $O/sys.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/torch -o c5 --output-format csv -- python3 tools/gpu/rt_first.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/torch.log 2>&1 || { tail -5 $O/torch.log; exit 1; }
echo ok
