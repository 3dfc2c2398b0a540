#!/bin/bash
# Round-4 closing measurements, part 2 (GPU box): the bench line with the
# committed r04 PMC counters folded in, C2 / C4 / C5 config lines and the
# N > 1 rehearsal (two ranks on the one GPU, the library sharding step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
P=profiles/r04_pmc
bash tools/gpu_steps.sh \
  bench_pmc 300 "python3 bench.py --steps 20 --warmup 5 --cpu-sample 256 --pmc-csv $P/fetch_r04_counter_collection.csv,$P/write_r04_counter_collection.csv > gpurun_out/r04_bench.json" \
  configs 700 "bash tools/configs_bench.sh" \
  rehearse 400 "python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --cpu-sample 0 --ragged-steps 0 --consumer-texts 0 > gpurun_out/rehearse2.json"
