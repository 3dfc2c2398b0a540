#!/bin/bash
# Round-4 GPU step set: layer parity, the GPU suite, bench, phase stamps.
# Each step under its own limit; a timeout / abort ends the chain (tools/gpu_steps.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  layers 400 "python -u -m pytest tests/test_layer_parity.py -x -v -s --timeout 300 --timeout-method thread" \
  tests 600 "python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread --deselect tests/test_layer_parity.py" \
  stamps 120 "build/phase_stamps" \
  bench 300 "python -u bench.py --steps 10 --warmup 3 --host-runs 3 --cpu-sample 0 --consumer-texts 0"
