#!/bin/bash
# Round 6: FFN-down of small batches (K = 1536) on 12 waves x 4 rounds instead
# of 16 x 3 — bitwise against the closing library, then one-sentence latency
# (bert_eval, 16 / 128 tokens), alternating, 3 runs each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bitwise_libs.py build/libbert.so build/ab/ks12/libbert.so > gpurun_out/ks12_bitwise.log 2>&1 || { tail -20 gpurun_out/ks12_bitwise.log; exit 1; }
grep -E "bitwise|differ" gpurun_out/ks12_bitwise.log | tail -8
for rep in 1 2 3; do
  for lib in build/libbert.so build/ab/ks12/libbert.so; do
    echo -n "$lib "
    BERT_AMD_LIB=$lib timeout -k 10 120 python3 tools/latency_probe.py --runs 200 --configs 2048:0 --lengths 16,128 2>/dev/null | tail -1 || exit 1
  done
done
