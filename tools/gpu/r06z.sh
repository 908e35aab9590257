set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06z
mkdir -p $O
ZB_PHASES_LIBRARY=1 timeout -k 10 300 python3 -u bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/c5_sys.json 2> $O/c5_sys.err || exit 1
ZB_PHASES_LIBRARY=1 timeout -k 10 300 python3 -u tools/gpu/rt_first.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline > $O/c5_torch.json 2> $O/c5_torch.err || exit 1
echo ok
