cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  qs 60 "build/qkva_stamps 10 pc" \
  pct 300 "python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread -k 'producer_consumer or small_batches or golden_vectors'" \
  ab 300 "for c in 2 0 2 0; do BERT_AMD_QKVA_NTW=\$c python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --profile-steps 2 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1; python3 -c \"import json;d=json.load(open('gpurun_out/ab.json'));print('ntw=\$c', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})\"; done"
