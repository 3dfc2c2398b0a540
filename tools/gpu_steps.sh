#!/bin/bash
# Run named GPU steps in order; each under its own timeout; log to gpurun_out/<name>.log.
# A step that fails normally (e.g. pytest rc=1) does not stop the chain; a
# timeout / abort / segfault / kill (rc >= 124) ends it immediately.
#   tools/gpu_steps.sh name1 secs1 "cmd1" [name2 secs2 "cmd2" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export BERT_AMD_MODEL_DIR=${BERT_AMD_MODEL_DIR:-/tmp/bert_amd_models}
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  echo "[$(date +%T)] step $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] step $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping: $name ended with rc=$rc"; exit $rc; fi
done
exit 0
