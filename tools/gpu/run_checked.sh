#!/bin/bash
# The GPU suite under the guard-band build (libzbgpu_checked.so, zeebe_amd/csrc/zb_checked.hpp): every launch is
# synchronised and every allocation's guard bands scanned; a test fails on any out-of-bounds write. The trace file
# logs every allocation and launch (it names the kernel if a launch faults).
# usage (repo root, on the GPU box): bash tools/gpu/run_checked.sh [pytest -k expression]
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/checked
mkdir -p $O
rm -f $O/trace.log
K=()
[ -n "$1" ] && K=(-k "$1")
export ZB_CHECKED_LIBRARY=1 ZB_CHECKED_TRACE=$O/trace.log
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
grep -h "ZB_CHECKED" $O/pytest.log $O/trace.log | sort | uniq -c | head -40
gzip -f $O/trace.log
exit $rc
