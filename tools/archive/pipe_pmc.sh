#!/bin/bash
# PMC passes over the real pipeline (bench.py, one row group, one step) for one
# GEMM-path setting (development):
#   tools/pipe_pmc.sh <tag> [ENV=VALUE ...]     results under gpurun_out/pipepmc/<tag>/
# e.g. tools/pipe_pmc.sh f6 BERT_AMD_F6=1 ; tools/pipe_pmc.sh i8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=$1; shift
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp BERT_AMD_SPLIT=0 BERT_AMD_MODEL_DIR=${BERT_AMD_MODEL_DIR:-/tmp/bert_amd_models}
OUT=$PWD/gpurun_out/pipepmc/$TAG; mkdir -p "$OUT"
B="$PWD/bench.py"
ARGS="--steps 1 --warmup 1 --profile-steps 1 --cpu-sample 0 --ragged-steps 0 --host-runs 0"
# model file cached once outside the profiler
( cd /tmp && timeout -k 10 200 python3 "$B" $ARGS ) > "$OUT/plain.log" 2>&1 || { tail -5 "$OUT/plain.log"; exit 1; }
for p in "cyc:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE" \
         "ins:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" \
         "lds:SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_MFMA" \
         "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
  name=${p%%:*}; ctr=${p#*:}
  ( cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o p -- python3 "$B" $ARGS ) > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$TAG $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/$name.log"; exit $rc; }
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
exit 0
