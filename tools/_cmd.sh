cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_steps.sh \
  ab 600 "bash tools/lib_ab_rag.sh build/libbert.so build/var/cp1/libbert.so build/var/cp2/libbert.so"
