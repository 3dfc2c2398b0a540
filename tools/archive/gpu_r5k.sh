#!/bin/bash
# Round 5: static priority for the later-dispatched waves of FFN-up / FFN-down (A/B, 3 runs each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  prio_ab 600 "REPS=3 bash tools/lib_ab.sh '--steps 20 --warmup 5' build/var/base/libbert.so build/var/prio1/libbert.so"
