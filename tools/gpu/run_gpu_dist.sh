#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path on one GPU (--same-device): torch.distributed.run, gloo control
# plane, one engine per rank; C3 with 2M instances per rank
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out/dist
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --instances 2000000 --same-device --no-extras --no-cpu-baseline > gpurun_out/dist/c3_2rank.json 2> gpurun_out/dist/c3_2rank.err || { echo "dist failed"; tail -20 gpurun_out/dist/c3_2rank.err; exit 1; }
cut -c1-700 gpurun_out/dist/c3_2rank.json
