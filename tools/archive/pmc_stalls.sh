#!/bin/bash
# Stall-breakdown PMC pass (development): SQ wave-cycle buckets and MFMA busy
# per kernel over a short bench run.  Output: gpurun_out/stalls/
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/stalls
B="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --ragged-steps 0 --host-runs 0 --profile-steps 0 ${BENCH_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d gpurun_out/stalls/p1 -o p1 --output-format csv -- $B > gpurun_out/stalls/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/stalls/p2 -o p2 --output-format csv -- $B > gpurun_out/stalls/p2.log 2>&1 || exit 1
