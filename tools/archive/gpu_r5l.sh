#!/bin/bash
# Round 5: consumer path (bert_encode_batch) A/B, round-4 library vs this one,
# 3 runs each alternating; and this library with small_rows 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
M=/tmp/bert_amd_models/minilm_q4_0_s20250117_w0.05.gguf
mkdir -p /tmp/bert_amd_models
[ -f $M ] || python3 -c "import sys; sys.path.insert(0, 'embedding.cpp_amd'); import bertlib; bertlib.synth_model('$M', 'minilm', 'q4_0', seed=20250117, w_std=0.05)" || exit 1
for rep in 1 2 3; do
  for lib in build/var/r4/libbert.so build/libbert.so; do
    timeout -k 10 120 python3 tools/consumer_ab.py $lib $M || exit 1
  done
  BERT_AMD_SMALL_ROWS=0 timeout -k 10 120 python3 tools/consumer_ab.py build/libbert.so $M || exit 1
done
