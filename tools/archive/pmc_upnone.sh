#!/bin/bash
# PMC passes over one GEMM shape of tools/gemm_bench (development tool).
#   tools/pmc_upnone.sh [mode]   -> gpurun_out/pmcun/<pass>/...
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmcun; mkdir -p $OUT
for p in "clk:GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
         "ins:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "mix:SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT"; do
  name=${p%%:*}; ctr=${p#*:}
  ( cd /tmp && timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o gb -- $GRAFT_REPO_ROOT/build/gemm_bench 3 ${1:-upnone} ) > $OUT/$name.log 2>&1
  echo "$name rc=$?"
done
