#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 120 --timeout-method thread -k "int8" > gpurun_out/q4r_tests.log 2>&1; grep -E "int8|passed|failed|Error" gpurun_out/q4r_tests.log | head -20
timeout -k 5 60 build/i8_bench 20 up || exit 1
BERT_AMD_Q4R=0 timeout -k 5 60 build/i8_bench 20 up || exit 1
BERT_AMD_I8=1 timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/bench_q4r.json 2> gpurun_out/bench_q4r.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_q4r.json'));print(d['value'],{k:v['avg_us'] for k,v in d['kernels'].items()})"
