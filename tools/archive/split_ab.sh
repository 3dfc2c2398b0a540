#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
A="--steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0 --profile-steps 1"
for rep in 1 2 3; do
  for sp in 1 0; do
    BERT_AMD_SPLIT=$sp timeout -k 10 200 python3 bench.py $A > gpurun_out/sab.json 2> gpurun_out/sab.err || { tail -3 gpurun_out/sab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/sab.json'));r=d.get('ragged') or {};s=d.get('ragged_short') or {};print('split=$sp', d['value'], 'ragged', r.get('value'), 'short', s.get('value'), flush=True)" | tee -a gpurun_out/split_ab.log
  done
done
