#!/bin/bash
# Round 6: the GPU suite on the current library, the golden / build-order tests
# with Q4_1's scale products on the bf16 MFMA (BERT_AMD_Q41BF=1), and C5 /
# MiniLM Q4_1 timed with q41bf 0 / 1 (2 runs each, alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
COMMON="--cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
bash tools/gpu_steps.sh \
  suite 600 "$T -m gpu tests/" \
  q41golden 600 "BERT_AMD_Q41BF=1 $T -m gpu tests/test_gpu_parity.py -k 'golden_vectors or each_ggml_build or c5_vs_each or every_weight_type or batch_invariance or small_row or unfused'" || exit $?
for rep in 1 2; do
  for bf in 0 1; do
    BERT_AMD_Q41BF=$bf timeout -k 10 400 python3 bench.py --shape bge-large --ftype q4_1 --batch 1024 --seq 512 --steps 3 --warmup 1 --profile-steps 1 $COMMON > gpurun_out/c5_bf$bf.json 2> gpurun_out/c5_bf$bf.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c5_bf$bf.json'));print('c5 q41bf=$bf', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)" >> gpurun_out/q41_ab.log
    BERT_AMD_Q41BF=$bf timeout -k 10 200 python3 bench.py --shape minilm --ftype q4_1 --steps 10 --warmup 3 $COMMON > gpurun_out/m41_bf$bf.json 2> gpurun_out/m41_bf$bf.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/m41_bf$bf.json'));print('minilm q4_1 q41bf=$bf', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)" >> gpurun_out/q41_ab.log
  done
done
cat gpurun_out/q41_ab.log
