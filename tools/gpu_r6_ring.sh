#!/bin/bash
# Round 6: branch-free weight ring of the producer / consumer kernel's producers
# (exact vmcnt waits), ring lead 2 and 3 — bitwise against the previous library,
# then alternating headline runs (3 each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bitwise_libs.py build/ab/head/libbert.so build/libbert.so build/ab/ah3/libbert.so > gpurun_out/ring_bitwise.log 2>&1 || { tail -20 gpurun_out/ring_bitwise.log; exit 1; }
tail -6 gpurun_out/ring_bitwise.log
REPS=3 bash tools/lib_ab.sh "--steps 20 --warmup 5 --ragged-steps 5" build/libbert.so build/ab/ah3/libbert.so build/ab/head/libbert.so
