set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06u
mkdir -p $O
ZB_SYSRT=1 ZB_SCHED=spin timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/sys_spin.txt 2>&1 || exit 1
ZB_SYSRT=1 ZB_SCHED=yield timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/sys_yield.txt 2>&1 || exit 1
ZB_SYSRT=1 HSA_ENABLE_INTERRUPT=0 timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/sys_noint.txt 2>&1 || exit 1
ZB_SCHED=spin timeout -k 10 300 python3 -u tools/gpu/c5_calls.py 1000000 4 > $O/torch_spin.txt 2>&1 || exit 1
echo ok
