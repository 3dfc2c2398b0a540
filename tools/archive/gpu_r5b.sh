#!/bin/bash
# Round 5, second GPU pass: the producer / consumer kernel with one barrier per
# period (double-buffered V^T, Q / K released by an LDS count) — its parity
# tests, then a 3-run A/B against the round-5 start (build/var/base) and the
# FFN-down LN kernel without the two-tile pipeline (build/var/lnp0: no scratch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  pc_tests 600 "$T tests/test_gpu_parity.py -k 'producer_consumer or golden_vectors or packed_short or device_batch_reordered or small_batches or full_size or batch_invariance or fresh_context' tests/test_layer_parity.py -k 'c3_minilm_q4_0-fused'" \
  ab 900 "REPS=3 bash tools/lib_ab.sh '--steps 20 --warmup 5' build/var/base/libbert.so build/libbert.so build/var/lnp0/libbert.so"
