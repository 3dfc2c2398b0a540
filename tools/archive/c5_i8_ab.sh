cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c5ab
for cfg in "BERT_AMD_I8=up" "BERT_AMD_I8=all"; do
  env $cfg timeout -k 10 300 python3 bench.py --shape bge-large --ftype q4_1 --batch 1024 --seq 512 --steps 3 --warmup 1 --profile-steps 1 --cpu-sample 0 --host-runs 0 --ragged-steps 0 > gpurun_out/c5ab/$cfg.json 2> gpurun_out/c5ab/$cfg.err || exit 1
  python3 -c "import json,sys;d=json.load(open('gpurun_out/c5ab/$cfg.json'));print('$cfg', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
