set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $O/full_sys.json 2> $O/full_sys.err || { tail -5 $O/full_sys.err; exit 1; }
timeout -k 10 600 python3 -u tools/gpu/rt_first.py --no-cpu-baseline > $O/full_torch.json 2> $O/full_torch.err || { tail -5 $O/full_torch.err; exit 1; }
echo ok
