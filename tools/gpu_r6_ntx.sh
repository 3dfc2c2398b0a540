#!/bin/bash
# Round 6: the LN kernel's X rows stored nontemporal (option nt_x, default 1;
# not the last layer's) — bitwise against HEAD's library, the GPU suite, then
# headline runs alternating BERT_AMD_NT_X=1 / 0 on the same library (3 each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bitwise_libs.py build/ab/head/libbert.so build/libbert.so > gpurun_out/ntx_bitwise.log 2>&1 || { tail -20 gpurun_out/ntx_bitwise.log; exit 1; }
grep -c "bitwise equal" gpurun_out/ntx_bitwise.log
bash tools/gpu_steps.sh suite 600 "python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" || exit $?
grep -q " passed" gpurun_out/suite.log && ! grep -q -E " failed| error" gpurun_out/suite.log || { echo "tests failed"; tail -30 gpurun_out/suite.log; exit 1; }
tail -1 gpurun_out/suite.log
COMMON="--steps 20 --warmup 5 --ragged-steps 5 --cpu-sample 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0 --profile-steps 2"
for rep in 1 2 3; do
  for v in 1 0; do
    BERT_AMD_NT_X=$v timeout -k 10 300 python3 bench.py $COMMON > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d.get('ragged') or {};print('nt_x=$v', d['value'], d['ms_per_step'], 'ragged', r.get('value'), {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)"
  done
done
