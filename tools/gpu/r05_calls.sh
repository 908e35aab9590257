#!/bin/bash
# Round-5 host / device split of the C2 steady tick and the C5 step at HEAD: per-call wall vs kernel time
# (tools/gpu/steady_calls.py, tools/gpu/c5_calls.py), the measurement build's host time per part of zb_step, and a
# kernel trace of each bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r05_calls}
mkdir -p $O
timeout -k 10 300 python3 -u tools/gpu/steady_calls.py 8 > $O/steady_calls.txt 2>&1 || { tail -5 $O/steady_calls.txt; exit 1; }
tail -17 $O/steady_calls.txt
ZB_PHASES_LIBRARY=1 timeout -k 10 300 python3 -u tools/gpu/steady_calls.py 8 > $O/steady_phases.txt 2>&1 || { tail -5 $O/steady_phases.txt; exit 1; }
grep "step ms" $O/steady_phases.txt | tail -8
timeout -k 10 300 python3 -u tools/gpu/c5_calls.py > $O/c5_calls.txt 2>&1 || { tail -5 $O/c5_calls.txt; exit 1; }
tail -25 $O/c5_calls.txt
TAG=c2s_r05 BENCH_ARGS="--config c2 --steady" bash tools/gpu/prof_cfg.sh || exit 1
TAG=c5_r05 BENCH_ARGS="--config c5" bash tools/gpu/prof_cfg.sh || exit 1
