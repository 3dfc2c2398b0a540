#!/bin/bash
# Round 6: O-tail forms — bitwise test per library, then the headline per form
# (o_tail 1 for each library; the default library with o_tail 0), 3 runs each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k o_tail"
for lib in build/libbert.so build/ab/t2a3/libbert.so build/ab/t2a2/libbert.so; do
  BERT_AMD_LIB=$lib timeout -k 10 200 $T > gpurun_out/ot_test.log 2>&1 || { echo "test failed $lib"; tail -20 gpurun_out/ot_test.log; exit 1; }
  echo "$lib bitwise ok"
done
A="--steps 20 --warmup 5 --cpu-sample 0 --consumer-texts 0 --load-replicas 0 --host-runs 0 --ragged-steps 0 --latency-runs 0"
for rep in 1 2 3; do
  for cfg in "build/libbert.so 1" "build/ab/t2a3/libbert.so 1" "build/ab/t2a2/libbert.so 1" "build/libbert.so 0"; do
    set -- $cfg
    BERT_AMD_LIB=$1 BERT_AMD_O_TAIL=$2 timeout -k 10 200 python3 bench.py $A > gpurun_out/ot.json 2> gpurun_out/ot.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ot.json'));print('$1 o_tail=$2', d['value'], d['roofline']['frac'], {k: v['avg_us'] for k, v in d['kernels'].items()}, flush=True)" >> gpurun_out/otail2_ab.log
  done
done
cat gpurun_out/otail2_ab.log
