#!/bin/bash
# Round 5: the producer / consumer kernel inside the pipeline — phase stamps of
# the default, consumers-first and consumer-priority builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  ps_def 120 "BERT_AMD_LIB=build/var/stamps/libbert.so python3 tools/pipe_stamps.py" \
  ps_cf 120 "BERT_AMD_LIB=build/var/stampscf/libbert.so python3 tools/pipe_stamps.py pass1 pass2 store period" \
  ps_p1 120 "BERT_AMD_LIB=build/var/stampsp1/libbert.so python3 tools/pipe_stamps.py" \
  ps_def2 120 "BERT_AMD_LIB=build/var/stamps/libbert.so python3 tools/pipe_stamps.py"
