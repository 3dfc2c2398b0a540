cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  qs 60 "build/qkva_stamps pc" \
  al 120 "build/attn_long_time c5 && build/attn_long_time c4 && build/attn_long_stamps c5 3 && build/attn_long_stamps c4 3" \
  pct 300 "python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'producer_consumer or packed_short or small_batches'" \
  ab 400 "bash tools/opt_ab.sh 'X=1' 'BERT_AMD_QKVA_NTW=2'"
