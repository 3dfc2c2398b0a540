#!/bin/bash
# A/B of library variants selected by env (development): tools/ab_bench.sh "ENV=.. ENV2=.." ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  for rep in 1 2; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --cpu-sample 0 --consumer-texts 0 --steps 30 > gpurun_out/ab/r$i.json 2> gpurun_out/ab/r$i.err || { tail -5 gpurun_out/ab/r$i.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab/r$i.json'));print(sys.argv[1], d['value'], 'host', (d.get('host_api') or {}).get('value'), 'ragged', d.get('ragged',{}).get('value'), 'short', (d.get('ragged_short') or {}).get('value'), 'ragged_host', (d.get('ragged') or {}).get('host_api',{}).get('value'), {k:v['avg_us'] for k,v in d['kernels'].items()})" "$cfg"
  done
done
