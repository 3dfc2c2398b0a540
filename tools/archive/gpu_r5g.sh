#!/bin/bash
# Round 5: small-batch (32-row tile) GEMM forms — bitwise tests first, then the
# bench line (single-sentence latency), the bf16-part probe and the C5 A/B of the
# Q4_1 scale-product forms.  (Diagnostics: tools/gpu_r5f.sh's last steps.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
C5="--shape bge-large --ftype q4_1 --batch 1024 --seq 512 --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
bash tools/gpu_steps.sh \
  small_tests 400 "$T tests/test_gpu_parity.py -k 'small_row_tiles or batch_invariance or small_batches_unfused'" || exit $?
grep -q " passed" gpurun_out/small_tests.log && ! grep -q "FAILED\|Error" gpurun_out/small_tests.log || { echo "small tests not green: stopping"; exit 1; }
bash tools/gpu_steps.sh \
  bench 300 "python3 bench.py --steps 20 --warmup 5 --cpu-sample 64 > gpurun_out/r05b_bench.json" \
  probe_bf16 60 "build/mfma_bf16_split_probe 65536" \
  c5_def 200 "python3 bench.py $C5 > gpurun_out/c5_def.json" \
  c5_bf 200 "BERT_AMD_Q41BF=1 python3 bench.py $C5 > gpurun_out/c5_bf.json" \
  c5_bf_all 200 "BERT_AMD_I8=all BERT_AMD_Q41BF=1 python3 bench.py $C5 > gpurun_out/c5_bf_all.json"
