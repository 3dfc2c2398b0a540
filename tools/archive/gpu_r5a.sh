#!/bin/bash
# Round 5, first GPU pass: the GPU suite on the default library (one-barrier
# producer / consumer kernel), a 3-run A/B (round-5 start, default, consumer
# priority 1, FFN-down LN kernel without the two-tile pipeline), the bench
# line, then the C5 build-order comparison on the Q4_1 plain-C-fold variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  tests 600 "$T tests -m gpu -x" \
  save 30 "mkdir -p gpurun_out/r05_default && cp gpurun_out/layer_parity_*.json gpurun_out/variants_*.json gpurun_out/r05_default/" \
  ab 600 "REPS=3 bash tools/lib_ab.sh '--steps 20 --warmup 5' build/var/base/libbert.so build/libbert.so build/var/cprio1/libbert.so build/var/lnp0/libbert.so" \
  bench 300 "python3 bench.py --steps 20 --warmup 5 --cpu-sample 64 > gpurun_out/r05a_bench.json" \
  q41gen 400 "BERT_AMD_LIB=build/var/q41gen/libbert.so $T tests/test_gpu_parity.py -k 'c5_vs_each or gpu_vs_each_ggml_build' tests/test_layer_parity.py -k 'c5'"
