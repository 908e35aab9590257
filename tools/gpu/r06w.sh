set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 120 python3 -u tools/probe/launch_probe.py sys > $O/sys.txt 2>&1 || exit 1
timeout -k 10 120 python3 -u tools/probe/launch_probe.py torch > $O/torch.txt 2>&1 || exit 1
echo ok
