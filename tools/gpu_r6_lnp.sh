#!/bin/bash
# Round 6: epilogue parameters (bias / LN weight / LN bias) staged in LDS in the
# int8 FFN-up and LN kernels — bitwise against the previous library, the GPU
# tests they touch, then alternating headline runs (3 each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bitwise_libs.py build/libbert.so build/ab/head/libbert.so > gpurun_out/lnp_bitwise.log 2>&1 || { tail -20 gpurun_out/lnp_bitwise.log; exit 1; }
tail -3 gpurun_out/lnp_bitwise.log
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh t 400 "$T tests/test_gpu_parity.py -k 'golden_vectors or small_row or batch_invariance or int8_gemm_path or producer_consumer or every_weight'" || exit $?
grep -q " passed" gpurun_out/t.log && ! grep -q -E " failed| error" gpurun_out/t.log || { echo "tests failed"; tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
REPS=3 bash tools/lib_ab.sh "--steps 20 --warmup 5 --ragged-steps 5" build/libbert.so build/ab/head/libbert.so
