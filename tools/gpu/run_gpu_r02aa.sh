#!/bin/bash
# tests + bench/prof (run_gpu_r02u.sh), then k_tmpl store experiments (ZB_TMPL_EXP 1: no log stores,
# 2: no srcd / vlen stores, 3: neither; the output is wrong, only the timing matters)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
RUN_TAG=${RUN_TAG:-r02aa} ./run_gpu_r02u.sh || exit 1
O=gpurun_out/${RUN_TAG:-r02aa}
for x in ${TEXPS:-1 2 3}; do
  ZB_TMPL_EXP=$x timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --no-drain --steps 3 > $O/texp$x.json 2> $O/texp$x.err || { echo "texp $x failed"; tail -5 $O/texp$x.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/texp$x.json')); r=d['roofline']; print('texp $x', r['kernel'], round(r['avg_launch_us'],1), 'us')"
done
