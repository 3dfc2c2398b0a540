#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 120 --timeout-method thread -k "golden_vectors or every_weight or int8 or fused_head" > gpurun_out/intw_tests.log 2>&1
rc=$?; grep -E "1-cos|passed|failed|Error" gpurun_out/intw_tests.log | head -30; [ $rc -ne 0 ] && exit $rc
BERT_AMD_I8=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 120 --timeout-method thread -k "golden_vectors and (c3 or q4_0)" > gpurun_out/intw_tests0.log 2>&1
rc=$?; grep -E "1-cos|passed|failed|Error" gpurun_out/intw_tests0.log | head -10; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh "X=1" "BERT_AMD_I8=0"
