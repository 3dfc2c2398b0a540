#!/bin/bash
# C5 (bge-large Q4_1, 512 tokens) A/B of the fused residual + LN GEMM
# (BERT_AMD_RESLN=1, default) against EPI_RESID + launch_ln (development).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B=${1:-256}
for v in 1 0 1 0; do
  BERT_AMD_RESLN=$v timeout -k 10 300 python3 bench.py --shape bge-large --ftype q4_1 --batch $B --seq 512 --steps 2 --warmup 1 \
    --profile-steps 1 --cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 > gpurun_out/c5_$v.json 2> gpurun_out/c5_$v.err || { tail -3 gpurun_out/c5_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c5_$v.json'));print('resln=$v', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
