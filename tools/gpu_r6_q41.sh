#!/bin/bash
# Round 6: the q41bf auto default (FFN-up on the bf16 scale products, the
# 384-wide FFN-down + LN kernel on the f32 MFMA): the GPU suite, then C5 and
# MiniLM Q4_1 bench lines with the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
COMMON="--cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
bash tools/gpu_steps.sh \
  suite 600 "$T -m gpu tests/" \
  c5 400 "python3 bench.py --shape bge-large --ftype q4_1 --batch 1024 --seq 512 --steps 3 --warmup 1 --profile-steps 1 $COMMON > gpurun_out/c5_auto.json" \
  m41 200 "python3 bench.py --shape minilm --ftype q4_1 --steps 10 --warmup 3 $COMMON > gpurun_out/m41_auto.json"
for f in c5_auto m41_auto; do python3 -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f', d['value'], d.get('dtype_note'), {k: v['avg_us'] for k, v in d['kernels'].items()})"; done
