cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  al 100 "build/attn_long_time c5 && build/attn_long_time c4" \
  tests 400 "python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k 'golden or ln_in_residual or mixed_lengths or batch_invariance or live_oracle or c5_north'" \
  c5 400 "bash tools/c5_now.sh build/libbert.so && BERT_AMD_LN_PASS=1 bash tools/c5_now.sh build/libbert.so"
