#!/bin/bash
# Round 6: producer / consumer role layout over the SIMDs (QKPC_LAYOUT) —
# bitwise against the default, then the A/B (3 runs each, alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  bitwise 300 "python3 -u tools/bitwise_libs.py build/libbert.so $*" || exit $?
if grep -q "DIFFERS" gpurun_out/bitwise.log; then echo "not bitwise: stop"; exit 1; fi
REPS=3 bash tools/lib_ab.sh '--steps 10 --warmup 3' build/libbert.so "$@"
