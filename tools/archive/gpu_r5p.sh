#!/bin/bash
# Round 5: faster WordPiece lookups — tokenizer / encode tests, then the consumer probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
bash tools/gpu_steps.sh \
  ttests 400 "$T tests/test_gpu_parity.py tests/test_tokenizer.py -k 'encode or consumer or token or server or golden_vectors'" || exit $?
grep -q " passed" gpurun_out/ttests.log && ! grep -q "FAILED\|Error" gpurun_out/ttests.log || { echo "tests not green: stopping"; exit 1; }
for rep in 1 2 3; do timeout -k 10 200 python3 tools/consumer_probe.py >> gpurun_out/consumer_probe3.log 2>&1 || exit 1; done
build/tok_bench /tmp/bert_amd_models/minilm_q4_0_s20250117_w0.05.gguf 4096 > gpurun_out/tok_bench_box.json
