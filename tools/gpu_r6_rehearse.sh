#!/bin/bash
# Round 6: the N > 1 bench path rehearsed on the one GPU of the box — 2 and 4
# ranks (torchrun, gloo barrier, every rank on device 0, the library's sharding
# over N replicas of device 0). The driver's scaling run uses one GPU per rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
A="--rehearse-one-gpu --steps 5 --warmup 2 --cpu-sample 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
bash tools/gpu_steps.sh \
  rehearse2 300 "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 $A > gpurun_out/rehearse2.json" \
  rehearse4 300 "python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 $A > gpurun_out/rehearse4.json"
