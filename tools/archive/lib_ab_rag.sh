#!/bin/bash
# Per-kernel A/B of library builds on the headline config, with the ragged lines (development):
#   tools/lib_ab_rag.sh lib1.so lib2.so ...   (each run twice, alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for rep in 1 2; do
  for lib in "$@"; do
    BERT_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 --ragged-steps 5 --consumer-texts 0 --profile-steps 2 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$lib'.split('/')[-2], d['value'], d['ms_per_step'], 'ragged', d['ragged']['value'], 'short', d['ragged_short']['value'], {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)"
  done
done
