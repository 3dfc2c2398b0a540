#!/bin/bash
# Fused vs unfused QKV + attention on the head-dim-64 shapes with 128-token
# sentences (development A/B; env BERT_AMD_UNFUSED=1 forces the unfused pair).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/d64
COMMON="--cpu-sample 0 --host-runs 0 --ragged-steps 0 --seq 128"
for cfg in "BERT_AMD_UNFUSED=1" "FUSED=1"; do
  env $cfg timeout -k 10 300 python3 bench.py --shape e5-base --ftype f16 --batch 1024 --steps 5 --warmup 2 $COMMON > gpurun_out/d64/e5_$cfg.json 2> gpurun_out/d64/e5_$cfg.err || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/d64/e5_$cfg.json'));print('e5 $cfg', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
  env $cfg timeout -k 10 300 python3 bench.py --shape bge-large --ftype q4_1 --batch 1024 --steps 3 --warmup 1 --profile-steps 1 $COMMON > gpurun_out/d64/bge_$cfg.json 2> gpurun_out/d64/bge_$cfg.err || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/d64/bge_$cfg.json'));print('bge $cfg', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
