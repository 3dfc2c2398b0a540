#!/bin/bash
# Round 5: bf16-part rounding probe, parity diagnostic (attention operand form),
# C5 A/B of the Q4_1 scale-product forms, and the bench line (latency breakdown).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
C5="--shape bge-large --ftype q4_1 --batch 1024 --seq 512 --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
bash tools/gpu_steps.sh \
  probe_bf16 60 "build/mfma_bf16_split_probe 65536" \
  c5_def 300 "python3 bench.py $C5 > gpurun_out/c5_def.json" \
  c5_bf 300 "BERT_AMD_Q41BF=1 python3 bench.py $C5 > gpurun_out/c5_bf.json" \
  c5_def_all 300 "BERT_AMD_I8=all python3 bench.py $C5 > gpurun_out/c5_def_all.json" \
  c5_bf_all 300 "BERT_AMD_I8=all BERT_AMD_Q41BF=1 python3 bench.py $C5 > gpurun_out/c5_bf_all.json" \
  q41tests 300 "$T tests/test_gpu_parity.py -k 'q41_bf16 or bf16_split'" \
  \
  diag_def 500 "BERT_AMD_PARITY_DIAG=1 $T tests/test_gpu_parity.py -k attention_operand_form tests/test_layer_parity.py -k c5" \
  save 30 "mkdir -p gpurun_out/diag_def && cp gpurun_out/layer_parity_*.json gpurun_out/attnform_*.json gpurun_out/diag_def/" \
  diag_gen 500 "BERT_AMD_PARITY_DIAG=1 BERT_AMD_LIB=build/var/q41gen/libbert.so $T tests/test_gpu_parity.py -k 'attention_operand_form and c5' tests/test_layer_parity.py -k c5"
