#!/bin/bash
# Per-kernel A/B of library builds on one config (development):
#   tools/lib_ab.sh "<bench.py args>" lib1.so lib2.so ...
# Each library runs REPS times (default 3), alternating, so that a kept /
# not-kept decision rests on >= 3 runs per side (DESIGN.md states the spread).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ARGS=$1; shift
REPS=${REPS:-3}
COMMON="--cpu-sample 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0 --profile-steps 2"
for rep in $(seq "$REPS"); do
  for lib in "$@"; do
    BERT_AMD_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS $COMMON > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d.get('ragged') or {};s=d.get('ragged_short') or {};print('${lib%/*}'.split('/')[-1], d['value'], d['ms_per_step'], 'ragged', r.get('value'), 'short', s.get('value'), {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)"
  done
done
