#!/bin/bash
# PMC passes over build/i8_bench (development): one rocprofv3 run per counter
# group (never more than the per-block slot limits), summaries under
# gpurun_out/pmci8/<group>.  Usage: tools/pmc_i8.sh [filter] [binary]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
BIN=$PWD/${2:-build/i8_bench}
OUT=$PWD/gpurun_out/pmci8; mkdir -p $OUT
for p in "cyc:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE" \
         "ins:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" \
         "lds:SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_MFMA"; do
  name=${p%%:*}; ctr=${p#*:}
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o i8 -- $BIN 3 ${1:-} ) > $OUT/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
