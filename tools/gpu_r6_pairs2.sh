#!/bin/bash
# Round 6: consumer pairs (QKPC_PAIRS) with soft_max's exp from the LDS table
# and in registers (QKPC_EXPREG) — bitwise against the default, stamps, A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  bitwise 300 "python3 -u tools/bitwise_libs.py build/libbert.so build/var/pairs1/libbert.so build/var/pairs_er/libbert.so" || exit $?
grep -q "DIFFERS" gpurun_out/bitwise.log && { echo "not bitwise: stop"; exit 1; }
echo "== pairs + register exp, consumer B detail"; STAMP_SLOTS=0,3,4,5,1,2 BERT_AMD_LIB=build/var/st2/libbert.so timeout -k 10 200 python3 tools/pipe_stamps.py scores+mxx exp waitA PV Xsync+store Y || exit 1
REPS=2 bash tools/lib_ab.sh '--steps 10 --warmup 3' build/libbert.so build/var/pairs1/libbert.so build/var/pairs_er/libbert.so
