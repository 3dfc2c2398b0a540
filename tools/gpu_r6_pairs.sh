#!/bin/bash
# Round 6: consumer pairs in the producer / consumer kernel (QKPC_PAIRS) —
# bitwise against the 4-consumer build, the kernel's GPU tests, then the A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  bitwise 300 "python3 -u tools/bitwise_libs.py build/var/pairs0/libbert.so build/libbert.so" \
  pctests 400 "$T -m gpu tests/test_gpu_parity.py -k 'producer or golden_vectors or batch_invariance or packed or fused or ragged'" || exit $?
grep -q "DIFFERS" gpurun_out/bitwise.log && { echo "not bitwise: stop"; exit 1; }
REPS=3 bash tools/lib_ab.sh '--steps 10 --warmup 3' build/var/pairs0/libbert.so build/libbert.so
