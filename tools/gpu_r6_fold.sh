cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  bitwise 400 "python3 -u tools/bitwise_libs.py build/libbert.so build/var/fold1/libbert.so build/var/fold2/libbert.so" \
  ab 900 "REPS=2 bash tools/lib_ab.sh '--steps 10 --warmup 3' build/libbert.so build/var/fold1/libbert.so build/var/fold2/libbert.so"
