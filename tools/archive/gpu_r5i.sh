#!/bin/bash
# Round 5: packed-fma fold A/B (I8_FOLD_W / I8_RES_FOLD_W variants), 3 runs each,
# alternating; then the bitwise small / batch tests on the default library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
bash tools/gpu_steps.sh \
  ftests 400 "$T tests/test_gpu_parity.py -k 'small_row_tiles or batch_invariance or producer_consumer or golden_vectors'" \
  fold_ab 800 "REPS=3 bash tools/lib_ab.sh '--steps 20 --warmup 5' build/var/fw1/libbert.so build/var/fw2/libbert.so build/var/fw2r1/libbert.so"
