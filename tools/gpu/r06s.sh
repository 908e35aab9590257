set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 6 > $O/c5_calls_torchrt.txt 2>&1 || exit 1
ZB_SYSRT=1 timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 6 > $O/c5_calls_sysrt.txt 2>&1 || exit 1
echo ok
