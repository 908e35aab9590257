#!/bin/bash
# GPU parity tests (one process), then smoke; every GPU step under its own time limit.
# usage (from the repo root, on the GPU box): bash tools/gpu/run_tests.sh [pytest -k expression]
set -o pipefail
O=gpurun_out/tests
mkdir -p $O
K=()
[ -n "$1" ] && K=(-k "$1")
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
