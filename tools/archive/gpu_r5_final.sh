#!/bin/bash
# Round 5, final library: the closing profile (bench line, kernel stats, PMC
# traffic; tools/profile_round.sh r05), the config lines, the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  profile 600 "bash tools/profile_round.sh r05" \
  configs 300 "CFG_OUT=gpurun_out/cfg bash tools/configs_bench.sh" \
  suite 600 "python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread"
