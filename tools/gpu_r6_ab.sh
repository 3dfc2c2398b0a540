#!/bin/bash
# Round 6: generic kernel-variant A/B — bitwise against the first library,
# then alternating bench runs (REPS each).
#   tools/gpu_r6_ab.sh base.so variant.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  bitwise 300 "python3 -u tools/bitwise_libs.py $*" || exit $?
if grep -q "DIFFERS" gpurun_out/bitwise.log; then echo "not bitwise: stop"; exit 1; fi
REPS=${REPS:-3} bash tools/lib_ab.sh '--steps 10 --warmup 3' "$@"
