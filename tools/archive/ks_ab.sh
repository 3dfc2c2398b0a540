#!/bin/bash
# Small-batch latency A/B (GPU box): the GPU small-row tests on build/libbert.so,
# then tools/latency_probe.py (small_rows 2048) on each library given, REPS
# alternating rounds.   tools/ks_ab.sh REPS lib1 lib2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
REPS=$1; shift
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "${KS_TESTS:-small_row_tiles or graph_replay or output_rows or batch_invariance or golden_vectors}" > gpurun_out/ks_tests.log 2>&1 || { tail -30 gpurun_out/ks_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/ks_tests.log
for r in $(seq "$REPS"); do
  for lib in "$@"; do
    echo -n "$lib " 
    BERT_AMD_LIB=$lib timeout -k 10 120 python tools/latency_probe.py --runs 200 --configs 2048:0 2>/dev/null | tail -1 || exit 1
  done
done
