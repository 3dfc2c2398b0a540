#!/bin/bash
# Round 6: int8 GEMMs' streamed activations (A chunks, residual tiles in;
# X / Q8 rows out) with the nontemporal cache policy (-DI8_NT=1), so the
# weights every tile re-reads stay in L2 — bitwise against HEAD, then
# alternating headline runs (3 each; PMC excess of down / O is the target).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bitwise_libs.py build/ab/head/libbert.so build/libbert.so build/ab/nt/libbert.so > gpurun_out/nt_bitwise.log 2>&1 || { tail -20 gpurun_out/nt_bitwise.log; exit 1; }
grep -E "bitwise|differ" gpurun_out/nt_bitwise.log | tail -16
REPS=3 bash tools/lib_ab.sh "--steps 20 --warmup 5 --ragged-steps 5" build/ab/nt/libbert.so build/ab/head/libbert.so build/libbert.so
