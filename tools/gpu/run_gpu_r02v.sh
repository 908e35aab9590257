#!/bin/bash
# drain write-pass bound experiments on C3 10M: ZB_SER_EXP 0 (full), 1 (no encode), 2 (no stream-out),
# 3 (neither), 4 (no header stores), 7 (only loads + scan)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
O=gpurun_out/${RUN_TAG:-r02v}
mkdir -p $O
for x in 0 1 2 3 4 7; do
  ZB_SER_EXP=$x timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 3 > $O/exp$x.json 2> $O/exp$x.err || { echo "exp $x failed"; tail -5 $O/exp$x.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/exp$x.json')); print('exp $x', round(d['step_breakdown_ms']['drain_write_kernel'],3), 'ms write pass')"
done
