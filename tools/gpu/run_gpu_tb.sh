#!/bin/bash
# GPU tests, then the full default bench line (extras + CPU baseline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
O=gpurun_out/${RUN_TAG:-tb}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 bench.py ${BENCH_ARGS} > $O/bench_full.json 2> $O/bench_full.err || { echo "full bench failed"; tail -20 $O/bench_full.err; exit 1; }
python3 - $O <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + '/bench_full.json'))
print(d['value'] / 1e9, d['ms_per_step'], d['roofline']['kernel'], round(d['roofline']['frac'], 3), d['step_breakdown_ms'])
for k, v in d.get('extras', {}).items():
    print(k, round(v['value'] / 1e9, 3), round(v['ms_per_step'], 2), 'stepping', round(v['stepping_ms'], 2), 'drain', round(v['drain_ms'], 2), [(o['kernel'][:60], round(o['avg_launch_us'], 1)) for o in v['roofline']['other_kernels']])
PY
