#!/bin/bash
# A/B of load-option settings through bench.py (development; env BERT_AMD_<KEY>
# is each load option's default): tools/opt_ab.sh "ENV=.. ENV2=.." ...  (each twice, alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 --ragged-steps 5 --consumer-texts 0 --profile-steps 2 > gpurun_out/ab/o.json 2> gpurun_out/ab/o.err || { tail -5 gpurun_out/ab/o.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab/o.json'));print(sys.argv[1], d['value'], d['ms_per_step'], 'ragged', d['ragged']['value'], 'short', d['ragged_short']['value'], {k:v['avg_us'] for k,v in d['kernels'].items()}, flush=True)" "$cfg"
  done
done
