cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  qs 90 "build/qkva_stamps 20 pc && build/var/qs_p4 20 pc" \
  pct 300 "python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'producer_consumer or packed_short or golden'" \
  pct4 300 "BERT_AMD_LIB=build/var/p4/libbert.so python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'producer_consumer or packed_short'" \
  ab 600 "bash tools/lib_ab.sh '--steps 20 --warmup 5' build/var/old/libbert.so build/libbert.so build/var/p4/libbert.so"
