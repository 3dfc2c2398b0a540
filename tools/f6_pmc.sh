#!/bin/bash
# Variant timing + PMC passes over the fp6 GEMM harness (development):
#   tools/f6_pmc.sh <filter> <binary> [binary...]   results under gpurun_out/f6pmc/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/f6pmc; mkdir -p $OUT
FILT=$1; shift
for b in "$@"; do
  echo "== $b"
  timeout -k 10 120 $PWD/$b 20 $FILT || exit $?
done
BIN=$PWD/$1
for p in "cyc:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE" \
         "ins:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" \
         "lds:SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_MFMA"; do
  name=${p%%:*}; ctr=${p#*:}
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o f6 -- $BIN 2 $FILT ) > $OUT/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py $OUT 2>/dev/null | head -40
exit 0
