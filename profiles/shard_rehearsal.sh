#!/bin/bash
# Rehearsal of bench.py's node-sharded mode on ONE GPU (every rank on GPU 0,
# gloo for the harness collectives): the mailbox exchange's per-pop device
# period with 2 ranks.  Usage (on the box, repo root): bash profiles/shard_rehearsal.sh <tag> [nodes pending]
set -o pipefail
TAG=${1:-r03}
N=${2:-100000}
P=${3:-800000}
cd ${GRAFT_REPO_ROOT:-.}
export KBHIP_BENCH_BACKEND=gloo KBHIP_BENCH_ONE_DEVICE=1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --nodes $N --pending $P \
    > gpurun_out/${TAG}_shard_rehearsal.json 2> gpurun_out/${TAG}_shard_rehearsal.err
