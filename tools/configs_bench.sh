#!/bin/bash
# Bench lines for the non-headline configurations (development; per-GPU shares
# of BASELINE configs 1, 3, 4).  Output: $OUT/*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT=${CFG_OUT:-gpurun_out/cfg}; mkdir -p $OUT
COMMON="--cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
timeout -k 10 200 python3 bench.py --shape minilm --ftype f16 --batch 256 --seq 128 --steps 20 $COMMON > $OUT/c2.json 2> $OUT/c2.err || exit 1
timeout -k 10 300 python3 bench.py --shape e5-base --ftype f16 --batch 512 --seq 256 --steps 5 --warmup 2 $COMMON > $OUT/c4.json 2> $OUT/c4.err || exit 1
timeout -k 10 400 python3 bench.py --shape bge-large --ftype q4_1 --batch 1024 --seq 512 --steps 3 --warmup 1 --profile-steps 1 $COMMON > $OUT/c5.json 2> $OUT/c5.err || exit 1
