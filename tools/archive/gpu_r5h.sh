#!/bin/bash
# Round 5: graph replay + small-tile bitwise tests, single-sentence latency A/B
# (tools/latency_probe.py) and its kernel trace (true kernel durations vs gaps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
bash tools/gpu_steps.sh \
  gtests 400 "$T tests/test_gpu_parity.py -k 'graph_replay or small_row_tiles or batch_invariance'" || exit $?
grep -q " passed" gpurun_out/gtests.log && ! grep -q "FAILED\|Error" gpurun_out/gtests.log || { echo "tests not green: stopping"; exit 1; }
bash tools/gpu_steps.sh \
  lat 200 "python3 tools/latency_probe.py --runs 300 > gpurun_out/lat.json" \
  lat_trace 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/lat_prof -o lat -- python3 tools/latency_probe.py --runs 50 --configs 2048:8 --lengths 16"
