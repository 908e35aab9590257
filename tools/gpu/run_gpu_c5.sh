#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
O=gpurun_out/${RUN_TAG:-c5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 bench.py --config c5 --steps 3 --warmup 1 > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('C5', d['value']/1e6, 'M transitions/s', d['ms_per_step'], 'ms/step')"
timeout -k 10 300 python3 tools/c5_phases.py 2>&1 | grep step
