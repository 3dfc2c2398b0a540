#!/bin/bash
# Round 5: C5 (bge-large Q4_1, 1024 x 512) projection forms A/B, 3 runs each, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
C5="--shape bge-large --ftype q4_1 --batch 1024 --seq 512 --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
for rep in 1 2 3; do
  for spec in default up+qkv up+qkv+o all; do
    if [ $spec = default ]; then unset BERT_AMD_I8; else export BERT_AMD_I8=$spec; fi
    timeout -k 10 200 python3 bench.py $C5 > gpurun_out/c5ab.json 2> gpurun_out/c5ab.err || { tail -3 gpurun_out/c5ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c5ab.json'));print('$spec', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)" | tee -a gpurun_out/c5ab.log
  done
done
