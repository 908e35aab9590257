#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out/dbg
timeout -k 5 200 python3 tools/debug_tmpl_io.py probe 65 > gpurun_out/dbg/survey.txt 2>&1; echo "rc=$?"; cat gpurun_out/dbg/survey.txt | tail -12
