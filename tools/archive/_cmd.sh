cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && bash tools/gpu_r4_close.sh
