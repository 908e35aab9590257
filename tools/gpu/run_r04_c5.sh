#!/bin/bash
# The C5 evidence at HEAD: PMC pass (installed into profiles/r04 of this tree first), the bench line, the kernel
# statistics. Every GPU step under its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
TAG=c5_1000000 BENCH_ARGS="--config c5" PMC_SETS="FETCH_SIZE;WRITE_SIZE" bash tools/gpu/run_gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_c5_1000000 $O/pmc_c5_1000000.json > $O/pmc_c5_1000000.txt || exit 1
cp $O/pmc_c5_1000000.json $O/pmc_c5_1000000.txt profiles/r04/
timeout -k 10 400 python3 -u bench.py --config c5 --steps 5 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -5 $O/bench_c5.err; exit 1; }
tail -1 $O/bench_c5.json | cut -c1-300
TAG=c5 BENCH_ARGS="--config c5" bash tools/gpu/prof_cfg.sh || exit 1
