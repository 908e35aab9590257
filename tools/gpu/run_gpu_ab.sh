#!/bin/bash
# same-box A/B of environment knobs on the C3 bench: AB_VARS="ZB_SER_LENBUF=0;ZB_SER_LENBUF=1" (each run twice)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
O=gpurun_out/${RUN_TAG:-ab}
mkdir -p $O
IFS=';' read -ra VS <<< "${AB_VARS}"
for rep in 1 2; do
  k=0
  for v in "${VS[@]}"; do
    k=$((k+1))
    env $v timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 5 ${BENCH_ARGS} > $O/ab${k}_$rep.json 2> $O/ab${k}_$rep.err || { echo "run $v failed"; tail -5 $O/ab${k}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab${k}_$rep.json')); b=d['step_breakdown_ms']; print('$v', round(d['ms_per_step'],3), 'ms/step', {k: round(x,3) for k,x in b.items()})"
  done
done
