#!/bin/bash
# Round 6: LayerNorm on read (batched two-rows-per-wave form) — its bitwise
# tests, then the single-sentence latency with ln_read 1 / 0 (3 runs each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh lnt 400 "$T tests/test_gpu_parity.py -k 'ln_on_read or small_row or batch_invariance or golden_vectors or graph_replay or unfused'" || exit $?
grep -q " passed" gpurun_out/lnt.log && ! grep -q -E " failed| error" gpurun_out/lnt.log || { echo "tests failed"; tail -30 gpurun_out/lnt.log; exit 1; }
tail -2 gpurun_out/lnt.log
A="--steps 5 --warmup 2 --profile-steps 1 --cpu-sample 0 --consumer-texts 0 --load-replicas 0 --host-runs 0 --ragged-steps 0"
for rep in 1 2 3; do
  for lr in 1 0; do
    BERT_AMD_LN_READ=$lr timeout -k 10 200 python3 bench.py $A > gpurun_out/lr$lr.json 2> gpurun_out/lr$lr.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/lr$lr.json'));print('ln_read=$lr', d['value'], {n: (v['us_median'], v['launches_per_call'], v['device_us']) for n, v in d['latency'].items() if n != 'note'}, flush=True)" >> gpurun_out/lnread2_ab.log
  done
done
cat gpurun_out/lnread2_ab.log
python3 -c "import json;d=json.load(open('gpurun_out/lr1.json'));print(json.dumps(d['latency']))"
