cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  pct 300 "python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'producer_consumer or packed_short or golden or batch_invariance'" \
  ab 300 "bash tools/lib_ab_rag.sh build/var/old/libbert.so build/libbert.so" && bash tools/gpu_r4_close.sh
