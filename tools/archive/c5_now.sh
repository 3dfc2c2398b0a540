#!/bin/bash
# C5 (bge-large Q4_1, 24 layers, 512 tokens) per-kernel times with a given
# library (development A/B): tools/c5_now.sh <lib.so> [batch]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B=${2:-256}
BERT_AMD_LIB=$1 timeout -k 10 400 python3 bench.py --shape bge-large --ftype q4_1 --batch $B --seq 512 --steps 2 --warmup 1 \
  --profile-steps 1 --cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 > /tmp/c5.json 2> /tmp/c5.err || { tail -3 /tmp/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('/tmp/c5.json'));print('$1'.split('/')[-1], d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
