#!/bin/bash
# Per-kernel times of the pipeline (bench.py's HIP-event pass, BERT_AMD_F6=1)
# for each ablation library build/abl/libbert_<bits>.so (development)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export BERT_AMD_F6=${BERT_AMD_F6:-1} TMPDIR=/tmp
mkdir -p gpurun_out/abl
for a in "$@"; do
  BERT_AMD_LIB=$PWD/build/abl/libbert_$a.so timeout -k 10 150 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 \
      --ragged-steps 0 --host-runs 0 --consumer-texts 0 > gpurun_out/abl/b_$a.log 2>&1 || { echo "abl $a failed"; tail -3 gpurun_out/abl/b_$a.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/abl/b_$a.log').read().strip().splitlines()[-1])
print('abl $a', d['ms_per_step'], {k: v.get('avg_us') for k, v in d.get('kernels', {}).items() if 'gemm' in k or 'qkv' in k})"
done
