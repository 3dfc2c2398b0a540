#!/bin/bash
# One round's measurement set on the GPU box (run from the repo root):
#   bench.py (with CPU baseline), rocprofv3 kernel-trace stats, FETCH_SIZE and
#   WRITE_SIZE counter passes, then bench.py again with the PMC traffic folded
#   into its roofline object.  Results under gpurun_out/round/.
#   tools/profile_round.sh <tag>
TAG=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp BERT_AMD_MODEL_DIR=${BERT_AMD_MODEL_DIR:-/tmp/bert_amd_models}
OUT=$PWD/gpurun_out/round
mkdir -p "$OUT"
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name"
  ( cd /tmp && timeout -k 10 "$secs" "$@" ) > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
}
B="$PWD/bench.py"
step bench 600 python3 "$B" --steps 20 --warmup 5 --cpu-sample 256
# kernel stats and counters per whole-batch launch (one row group; bench.py's own
# event pass does the same), so rocprofv3 averages match the bench's roofline
export BERT_AMD_SPLIT=0
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o $TAG -- python3 "$B" --steps 10 --warmup 3 --cpu-sample 0 --ragged-steps 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0
step fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o $TAG -- python3 "$B" --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --ragged-steps 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0
step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o $TAG -- python3 "$B" --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 --ragged-steps 0 --host-runs 0 --consumer-texts 0 --latency-runs 0 --load-replicas 0
F=$(find "$OUT/fetch" -name '*counter_collection.csv' | head -1)
W=$(find "$OUT/write" -name '*counter_collection.csv' | head -1)
python3 tools/hbm_summary.py "$OUT/fetch" "$OUT/write" "$TAG bench (C3 minilm q4_0 1024x128)" > "$OUT/${TAG}_pmc_hbm.txt"
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "minilm q4_0 batch=1024 seq_len=128" "$OUT/pmc_traffic.json" \
    "$TAG, tools/profile_round.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py"
cp "$(find "$OUT/stats" -name '*kernel_stats.csv' | head -1)" "$OUT/${TAG}_kernel_stats.csv"
unset BERT_AMD_SPLIT
step bench_pmc 600 python3 "$B" --steps 20 --warmup 5 --cpu-sample 256 --pmc-csv "$F,$W"
tail -1 "$OUT/bench_pmc.log" > "$OUT/${TAG}_bench.json"
cat "$OUT/${TAG}_bench.json"
