#!/bin/bash
# Per-kernel A/B of library builds on one config (development):
#   tools/lib_ab.sh "<bench.py args>" lib1.so lib2.so ...   (each run twice, alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ARGS=$1; shift
COMMON="--cpu-sample 0 --host-runs 0 --ragged-steps 0 --consumer-texts 0 --profile-steps 1"
for rep in 1 2; do
  for lib in "$@"; do
    BERT_AMD_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS $COMMON > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('${lib##*/}', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)"
  done
done
