#!/bin/bash
# One-sentence latency A/B of a context option (GPU box): tools/latency_probe.py
# with --opts KEY=a and KEY=b, REPS alternating rounds.
#   tools/opt_latency_ab.sh REPS "k=v1" "k=v2" [probe args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
REPS=$1; A=$2; B=$3; shift 3
for r in $(seq "$REPS"); do
  for o in "$A" "$B"; do
    timeout -k 10 120 python tools/latency_probe.py --runs 300 --configs 2048:0 --opts "$o" "$@" 2>/dev/null | tail -1 || exit 1
  done
done
