#!/bin/bash
# Round-4 closing measurements, part 1 (GPU box): the GPU suite with the
# per-layer parity tables, then tools/profile_round.sh r04.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  tests 900 "python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  profile 1000 "bash tools/profile_round.sh r04"
