#!/bin/bash
# Round-4 closing measurement set in one GPU call: the GPU suite (with the
# per-layer parity tables), tools/profile_round.sh r04 (bench + rocprofv3 stats
# + FETCH_SIZE / WRITE_SIZE passes + the bench line with the counters), the
# C2 / C4 / C5 config lines and the two-rank rehearsal of the N > 1 path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  tests 420 "python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  profile 600 "bash tools/profile_round.sh r04" \
  configs 300 "bash tools/configs_bench.sh" \
  rehearse 200 "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --cpu-sample 0 --ragged-steps 0 --consumer-texts 0 > gpurun_out/rehearse2.json"
