#!/bin/bash
# A/B sweep of one environment variable over the C3 headline bench line (no extras, no CPU baseline).
# usage: VAR=ZB_X VALUES="a b c" BENCH_ARGS="..." bash tools/gpu/sweep_env.sh
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/sweep_${VAR}
mkdir -p $O
for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 python3 bench.py --no-extras --no-cpu-baseline --steps 5 ${BENCH_ARGS} > $O/$v.json 2> $O/$v.err || { echo "$v failed"; tail -5 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.json')); b=d['step_breakdown_ms']; print('$VAR=$v', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', {k: round(x,3) for k,x in b.items()})"
done
