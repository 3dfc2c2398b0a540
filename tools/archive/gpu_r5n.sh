#!/bin/bash
# Round 5: what bounds the pipeline's kernels — SQ issue / wait counters and the
# effective clock per kernel (rocprofv3 --pmc, one pass per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp BERT_AMD_SPLIT=0
R=$GRAFT_REPO_ROOT
A="--steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --ragged-steps 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*\|GRBM_[A-Z_]*" $R/gpurun_out/counters_list.txt | sort -u > $R/gpurun_out/counters_names.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/sqa -o sqa -- python3 $R/bench.py $A > $R/gpurun_out/sqa.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAVES --output-format csv -d $R/gpurun_out/sqb -o sqb -- python3 $R/bench.py $A > $R/gpurun_out/sqb.log 2>&1
echo "rc=$?"
