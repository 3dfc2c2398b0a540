#!/bin/bash
# Round-5 closing measurements (GPU box): the rocprofv3 kernel summary, PMC
# FETCH / WRITE passes and the bench line with that traffic folded in
# (tools/profile_round.sh r05), the C2 / C4 / C5 config lines, and the N > 1
# rehearsal (two ranks on the one GPU, the library sharding step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  profile 900 "bash tools/profile_round.sh r05" \
  configs 700 "CFG_OUT=gpurun_out/cfg bash tools/configs_bench.sh" \
  rehearse 400 "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --cpu-sample 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0 > gpurun_out/rehearse2.json"
