set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 300 python3 -u tools/gpu/rt_first.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_torchrt.json 2> $O/c5_torchrt.err || exit 1
timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_sysrt.json 2> $O/c5_sysrt.err || exit 1
timeout -k 10 300 python3 -u tools/gpu/rt_first.py --steps 10 --warmup 2 --no-extras --no-cpu-baseline > $O/c3_torchrt.json 2> $O/c3_torchrt.err || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-extras --no-cpu-baseline > $O/c3_sysrt.json 2> $O/c3_sysrt.err || exit 1
timeout -k 10 300 python3 -u tools/gpu/rt_first.py --config c2 --steps 5 --warmup 1 --no-extras --no-cpu-baseline > $O/c2_torchrt.json 2> $O/c2_torchrt.err || exit 1
timeout -k 10 300 python3 -u bench.py --config c2 --steps 5 --warmup 1 --no-extras --no-cpu-baseline > $O/c2_sysrt.json 2> $O/c2_sysrt.err || exit 1
echo ok
