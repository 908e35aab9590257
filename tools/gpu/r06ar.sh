set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ar
mkdir -p $O
# tiles claimed from a counter (k_wave) against round-robin tiles: same-box A/B of C2 / C4 wave-only stepping
LIBS="ab/head.so ab/claim.so" REPS=2 OUT=$O/ab bash tools/gpu/wave_ab.sh || exit 1
# the 8-partition C4 run on this one GPU (eight ranks sharing it) with the claiming library
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29521 bench.py --config c4 --gpus 8 --same-device --instances 125000 --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/c4_8rank.json 2> $O/c4_8rank.err || { echo "c4 8-rank failed"; tail -20 $O/c4_8rank.err; exit 1; }
cat $O/c4_8rank.json
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "wave or trajectory or c4 or cancel or boundary" > $O/pytest_wave.log 2>&1 || { tail -30 $O/pytest_wave.log; exit 1; }
tail -3 $O/pytest_wave.log
echo ok
