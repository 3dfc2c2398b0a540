#!/bin/bash
# Round 6 final measurements on the closing library: the GPU suite, smoke, the
# round profile (bench line, rocprofv3 kernel summary, PMC FETCH / WRITE
# passes), the SQ issue / wait counters of the four big kernels
# (tools/sq_counters.py) and the C2 / C4 / C5 lines.  Two calls (gpurun's
# limit): tools/gpu_r6_final.sh 1, then tools/gpu_r6_final.sh 2 (tools/sq_counters.py
# then runs in the container on both calls' merged results).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
A="--steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --ragged-steps 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0"
if [ "$1" = "1" ]; then
bash tools/gpu_steps.sh \
  suite 600 "$T -m gpu tests/" \
  smoke 200 "python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  profile 700 "bash tools/profile_round.sh r06" || exit $?
exit 0
fi
# second call: the counters and the other configurations
bash tools/gpu_steps.sh \
  sqa 120 "cd /tmp && BERT_AMD_SPLIT=0 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/sqa -o sqa -- python3 $R/bench.py $A" \
  sqb 120 "cd /tmp && BERT_AMD_SPLIT=0 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAVES --output-format csv -d $R/gpurun_out/sqb -o sqb -- python3 $R/bench.py $A" \
  configs 600 "CFG_OUT=gpurun_out/cfg bash tools/configs_bench.sh" || exit $?
exit 0
# then, in the container (gpurun_out/ holds both calls' merged results):
#   python3 tools/sq_counters.py gpurun_out/sqa gpurun_out/sqb gpurun_out/round/r06_kernel_stats.csv \
#     profiles/r06_sq_counters.json "<source>"
