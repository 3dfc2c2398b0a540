#!/bin/bash
# Round 6: rocprofv3 kernel trace of the server path (bert_eval on one
# sentence of 16 and of 128 tokens, the default small-batch options) on the
# final library; tools/archive/last_call_kernels.py turns the CSV into the
# per-kernel sequence of the last call (run here, after the merge).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  lat16 200 "cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lat16 -o lat16 -- python3 $R/tools/latency_probe.py --runs 30 --configs 2048:0 --lengths 16" \
  lat128 200 "cd /tmp && rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lat128 -o lat128 -- python3 $R/tools/latency_probe.py --runs 30 --configs 2048:0 --lengths 128"
