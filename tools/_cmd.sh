cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  pct 300 "python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'producer_consumer or packed_short or golden'" \
  ab 600 "bash tools/lib_ab_rag.sh build/var/old/libbert.so build/libbert.so build/var/ah3/libbert.so"
