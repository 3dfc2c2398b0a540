#!/bin/bash
# Round 5 parity diagnostic: the GPU against the oracle with ggml's attention
# and with the GPU kernels' attention operand form, end to end and per layer,
# on the default library and on the Q4_1 plain-C-fold variant (build/var/q41gen).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp BERT_AMD_PARITY_DIAG=1
T="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
bash tools/gpu_steps.sh \
  probe_bf16 60 "build/mfma_bf16_split_probe 65536" \
  diag_def 500 "$T tests/test_gpu_parity.py -k attention_operand_form tests/test_layer_parity.py -k c5" \
  save 30 "mkdir -p gpurun_out/diag_def && cp gpurun_out/layer_parity_*.json gpurun_out/attnform_*.json gpurun_out/diag_def/" \
  diag_gen 500 "BERT_AMD_LIB=build/var/q41gen/libbert.so $T tests/test_gpu_parity.py -k 'attention_operand_form and c5' tests/test_layer_parity.py -k c5"
