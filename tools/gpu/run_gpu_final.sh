#!/bin/bash
# smoke, GPU tests, full default bench line (extras + CPU baseline), C5 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
O=gpurun_out/${RUN_TAG:-final}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
RUN_TAG=${RUN_TAG:-final} ./run_gpu_tb.sh || exit 1
timeout -k 10 300 python3 bench.py --config c5 --steps 3 --warmup 1 > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('C5', d['value']/1e6, 'M transitions/s', d['ms_per_step'], 'ms/step')"
