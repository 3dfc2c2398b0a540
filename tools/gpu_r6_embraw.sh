#!/bin/bash
# Round 6: the word-embedding table in its GGUF row format (option emb_raw) —
# bitwise against the f32 copy (F16 / Q4_0 / Q4_1 models), then the A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
BITWISE_FTYPES=f16,q4_0,q4_1 bash tools/gpu_steps.sh \
  bitwise 300 "python3 -u tools/bitwise_libs.py build/libbert.so build/libbert.so@BERT_AMD_EMB_RAW=1" || exit $?
grep -q "DIFFERS" gpurun_out/bitwise.log && { echo "not bitwise: stop"; exit 1; }
COMMON="--cpu-sample 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0 --profile-steps 2"
for rep in 1 2 3; do
  for er in 0 1; do
    BERT_AMD_EMB_RAW=$er timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 $COMMON > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d.get('ragged') or {};print('emb_raw=$er', d['value'], d['ms_per_step'], 'ragged', r.get('value'), {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)"
  done
done
