#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out/dbg
timeout -k 5 120 python3 tools/debug_tmpl_io.py 300 > gpurun_out/dbg/io300.txt 2>&1; echo "rc=$?"; head -30 gpurun_out/dbg/io300.txt
