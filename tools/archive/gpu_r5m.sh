#!/bin/bash
# Round 5: consumer-path host overheads (encode tokenisation buffers, permuted
# outputs written in place): bitwise tests, then the probe A/B against HEAD's
# library, 3 runs each alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 600 --timeout-method thread"
bash tools/gpu_steps.sh \
  etests 400 "$T tests/test_gpu_parity.py -k 'encode or consumer or batch_invariance or golden_vectors or small_row'" || exit $?
grep -q " passed" gpurun_out/etests.log && ! grep -q "FAILED\|Error" gpurun_out/etests.log || { echo "tests not green: stopping"; exit 1; }
for rep in 1 2 3; do
  for lib in build/var/head/libbert.so build/libbert.so; do
    BERT_AMD_LIB=$lib timeout -k 10 200 python3 tools/consumer_probe.py >> gpurun_out/consumer_probe_ab.log 2>&1 || exit 1
    echo "lib=$lib" >> gpurun_out/consumer_probe_ab.log
  done
done
