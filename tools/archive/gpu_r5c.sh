#!/bin/bash
# Round 5: phase stamps of the producer / consumer kernel, one barrier per
# period (build/qkva_stamps) vs the round-4 two-barrier form (build/qkva_stamps_base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_steps.sh \
  st_new 120 "build/qkva_stamps 20 pc" \
  st_base 120 "build/qkva_stamps_base 20 pc" \
  st_new2 120 "build/qkva_stamps 20 pc" \
  st_base2 120 "build/qkva_stamps_base 20 pc"
