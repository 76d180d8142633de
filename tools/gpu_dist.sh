#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: 2 ranks under torch.distributed.run,
# gloo for the timing barrier / max-over-ranks (RCCL needs one GPU per rank), both on cuda:0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
FMPNP_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --legs none --steps 500 --warmup 5 --batch 64 \
  > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { tail -30 gpurun_out/dist2.err; exit 1; }
tail -1 gpurun_out/dist2.json | cut -c1-400
FMPNP_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --legs none --steps 500 --warmup 5 --global-batch 128 \
  > gpurun_out/dist2s.json 2> gpurun_out/dist2s.err || { tail -30 gpurun_out/dist2s.err; exit 1; }
tail -1 gpurun_out/dist2s.json | cut -c1-400
