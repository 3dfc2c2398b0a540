cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  qs 60 "build/qkva_stamps 20 pc && build/var/qkva_stamps_p1 20 pc" \
  al 200 "for x in build/attn_long_time build/var/alt_prio build/var/alt_nk64 build/var/alt_nk64p build/attn_long_time build/var/alt_prio build/var/alt_nk64 build/var/alt_nk64p; do echo \$x; \$x c5 && \$x c4 || exit 1; done; build/attn_long_stamps c5 3 && build/var/als_nk64 c5 3" \
  tests 400 "python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k 'golden or ln_in_residual or mixed_lengths or batch_invariance or live_oracle'" \
  c5 400 "bash tools/c5_now.sh build/libbert.so && BERT_AMD_LN_PASS=1 bash tools/c5_now.sh build/libbert.so" \
  ab 500 "bash tools/lib_ab.sh '--steps 20 --warmup 5' build/libbert.so build/var/cp1/libbert.so build/var/cp2/libbert.so build/var/cp3/libbert.so"
