#!/bin/bash
# Round 6: the O tail of qkv_attention_pc_kernel — its bitwise test against the
# separate O + LN launch, the suites it touches, then the headline with
# o_tail 1 / 0 (2 runs each, alternating) and the latency line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
A="--steps 20 --warmup 5 --cpu-sample 0 --consumer-texts 0 --load-replicas 0 --host-runs 0 --ragged-steps 0"
bash tools/gpu_steps.sh \
  otail 400 "$T -m gpu tests/test_gpu_parity.py -k 'o_tail or producer_consumer or golden_vectors or small_row or batch_invariance or int8_gemm_path'" || exit $?
grep -q " passed" gpurun_out/otail.log && ! grep -q " failed" gpurun_out/otail.log || { echo "tests failed"; exit 1; }
for rep in 1 2; do
  for ot in 1 0; do
    BERT_AMD_O_TAIL=$ot timeout -k 10 200 python3 bench.py $A > gpurun_out/ot$ot.json 2> gpurun_out/ot$ot.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ot$ot.json'));print('o_tail=$ot', d['value'], d['roofline']['frac'], {k: v['avg_us'] for k, v in d['kernels'].items()}, {n: v['us_median'] for n, v in d['latency'].items() if n != 'note'}, flush=True)" >> gpurun_out/otail_ab.log
  done
done
cat gpurun_out/otail_ab.log
