set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06ao
mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --same-device --instances 2000000 --steps 3 --warmup 1 > $O/bench_2rank.json 2> $O/bench_2rank.err || { echo "2-rank failed"; tail -20 $O/bench_2rank.err; exit 1; }
echo ok
