#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/q4rprof; export TMPDIR=/tmp
OUT=$PWD/gpurun_out/q4rprof; BIN=$PWD/build/i8_bench
( cd /tmp && timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o s -- $BIN 5 up ) > $OUT/stats.log 2>&1 || exit 1
for p in "cyc:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE" \
         "ins:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM" \
         "act:SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  name=${p%%:*}; ctr=${p#*:}
  ( cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o i8 -- $BIN 3 up ) > $OUT/$name.log 2>&1 || exit 1
done
