#!/bin/bash
# PMC passes over q4r ablation builds (development): tools/q4r_pmc.sh e1 e2 ...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for e in "$@"; do
  OUT=$PWD/gpurun_out/q4rpmc/e$e; mkdir -p $OUT
  for p in "cyc:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "ins:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA"; do
    name=${p%%:*}; ctr=${p#*:}
    ( cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$name -o q -- $GRAFT_REPO_ROOT/build/q4r_e$e 3 up ) > $OUT/$name.log 2>&1 || exit 1
  done
done
