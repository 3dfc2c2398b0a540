#!/bin/bash
# Round 5: the attention-operand-form parity diagnostic on the GPU:
# GPU vs the oracle with ggml's attention and with the GPU's operand form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 900 --timeout-method thread"
bash tools/gpu_steps.sh \
  diag_def 1000 "BERT_AMD_PARITY_DIAG=1 $T tests/test_gpu_parity.py -k attention_operand_form"
