set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06t
mkdir -p $O
ZB_SYSRT=1 HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/sys_kern0.txt 2>&1 || exit 1
ZB_SYSRT=1 HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/sys_kern1.txt 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/torch_kern1.txt 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/torch_kern0.txt 2>&1 || exit 1
echo ok
