#!/bin/bash
# Round 6: nontemporal STORES only (no nt loads) on the int8 GEMMs' outputs:
# st1 = X rows + Q8 rows (-DI8_NT_ST=1), st2 = the LN kernel's X rows only
# (-DI8_NT_ST=2) — bitwise against HEAD, then alternating headline runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bitwise_libs.py build/ab/head/libbert.so build/ab/st1/libbert.so build/ab/st2/libbert.so > gpurun_out/ntst_bitwise.log 2>&1 || { tail -20 gpurun_out/ntst_bitwise.log; exit 1; }
grep -c "bitwise equal" gpurun_out/ntst_bitwise.log
REPS=3 bash tools/lib_ab.sh "--steps 20 --warmup 5 --ragged-steps 5" build/ab/st1/libbert.so build/ab/st2/libbert.so build/ab/head/libbert.so
