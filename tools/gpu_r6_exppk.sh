#!/bin/bash
# Round 6: the fused kernel's softmax lookups two scores at a time (packed fp16
# conversion + packed clamp, table at a fixed LDS offset) — bitwise against the
# previous library, the fused-kernel GPU tests, then alternating headline runs
# (3 each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bitwise_libs.py build/ab/head/libbert.so build/libbert.so > gpurun_out/exppk_bitwise.log 2>&1 || { tail -20 gpurun_out/exppk_bitwise.log; exit 1; }
tail -4 gpurun_out/exppk_bitwise.log
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh t 400 "$T tests/test_gpu_parity.py -k 'golden_vectors or batch_invariance or producer_consumer or packed or fused'" || exit $?
grep -q " passed" gpurun_out/t.log && ! grep -q -E " failed| error" gpurun_out/t.log || { echo "tests failed"; tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
REPS=3 bash tools/lib_ab.sh "--steps 20 --warmup 5 --ragged-steps 5" build/libbert.so build/ab/head/libbert.so
