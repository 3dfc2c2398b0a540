#!/bin/bash
# A/B of the host-API (bert_eval_batch) rate between two library builds (development)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hab
for i in 1 2 3; do for cfg in BERT_AMD_LIB=build/abbase/libbert.so X=new; do
 env $cfg timeout -k 10 200 python bench.py --cpu-sample 0 --steps 10 --warmup 3 --host-runs 20 > gpurun_out/hab/$i.json 2>/dev/null || exit 1
 python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['host_api']['ms_median'], d['host_api']['ms_min'], d['ragged']['value'], d['ragged']['host_api']['ms_median'])" gpurun_out/hab/$i.json $cfg
done; done
