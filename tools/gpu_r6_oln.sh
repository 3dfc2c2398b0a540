#!/bin/bash
# Round 6: small-batch O + residual as 64-column tiles + the LN rows kernel
# (option small_oln) — bitwise against the 384-wide O + LN tile, the small-row
# GPU tests, then the single-sentence latency A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
[ "$1" = ab ] || BITWISE_FTYPES=f16,q4_0,q4_1 bash tools/gpu_steps.sh \
  bitwise 300 "python3 -u tools/bitwise_libs.py build/libbert.so@BERT_AMD_SMALL_OLN=0 build/libbert.so@BERT_AMD_SMALL_OLN=1" \
  smalltests 400 "$T -m gpu tests/test_gpu_parity.py -k 'small_row or batch_invariance or unfused or golden_vectors'" || exit $?
if [ "$1" != ab ] && grep -q "DIFFERS" gpurun_out/bitwise.log; then echo "not bitwise: stop"; exit 1; fi
COMMON="--cpu-sample 0 --host-runs 0 --consumer-texts 0 --ragged-steps 0 --load-replicas 0 --steps 3 --warmup 1 --profile-steps 1"
for rep in 1 2 3; do
  for v in 0 1; do
    BERT_AMD_SMALL_OLN=$v timeout -k 10 300 python3 bench.py $COMMON > gpurun_out/lat.json 2> gpurun_out/lat.err || { tail -3 gpurun_out/lat.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/lat.json'));l=d['latency'];print('small_oln=$v', d['value'], {k: (v['us_median'], v['launches_per_call'], v['kernel_us']) for k, v in l.items() if k in ('n16', 'n32', 'n128')}, flush=True)"
  done
done
