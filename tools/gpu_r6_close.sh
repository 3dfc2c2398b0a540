#!/bin/bash
# Round 6 closing measurements on the GPU box: the GPU suite, smoke, the round
# profile (bench line, rocprofv3 kernel summary, PMC FETCH / WRITE passes) and
# the C2 / C4 / C5 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  suite 600 "$T -m gpu tests/" \
  smoke 200 "python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  profile 1000 "bash tools/profile_round.sh r06" \
  configs 900 "CFG_OUT=gpurun_out/cfg bash tools/configs_bench.sh"
