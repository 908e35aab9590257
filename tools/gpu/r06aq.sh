set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06aq
mkdir -p $O
# C4 with P = 8 partitions (one engine per rank, eight ranks sharing the one GPU of this box: the partitions are
# independent, so this runs the 8-partition configuration, not its scaling)
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29521 bench.py --config c4 --gpus 8 --same-device --instances 125000 --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/c4_8rank.json 2> $O/c4_8rank.err || { echo "c4 8-rank failed"; tail -20 $O/c4_8rank.err; exit 1; }
echo ok
