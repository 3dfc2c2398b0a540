#!/bin/bash
# Round 6: C5 (bge-large Q4_1, 1024 x 512) projection forms re-measured with
# the q41bf auto default (int8 projections other than the 384-wide FFN-down +
# LN take Q4_1's scale products on the bf16 MFMA): i8 = up (default at n_embd
# 1024), up+down, o+up+down, all.  Two runs per form, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
COMMON="--cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
for rep in 1 2; do
  for form in up up+down o+up+down all; do
    BERT_AMD_I8=$form timeout -k 10 300 python3 bench.py --shape bge-large --ftype q4_1 --batch 1024 --seq 512 \
      --steps 3 --warmup 1 --profile-steps 1 $COMMON > gpurun_out/c5f.json 2> gpurun_out/c5f.err || { tail -5 gpurun_out/c5f.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c5f.json'));print('$form', d['value'], d['ms_per_step'], d.get('dtype_note'), {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)"
  done
done
