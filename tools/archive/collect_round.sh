#!/bin/bash
# After tools/gpu_r4_close.sh (its gpurun_out/ merged back here): copy the
# round's measurement records into profiles/ (run in this container).
#   tools/collect_round.sh r04
TAG=${1:-r04}
cd "$(dirname "$0")/.." || exit 2
R=gpurun_out/round
set -e
mkdir -p profiles/${TAG}_pmc
cp $R/${TAG}_kernel_stats.csv $R/${TAG}_pmc_hbm.txt profiles/
cp $R/fetch/${TAG}_counter_collection.csv profiles/${TAG}_pmc/fetch_${TAG}_counter_collection.csv
cp $R/write/${TAG}_counter_collection.csv profiles/${TAG}_pmc/write_${TAG}_counter_collection.csv
python3 tools/pmc_traffic.py $R/fetch $R/write "minilm q4_0 batch=1024 seq_len=128" profiles/pmc_traffic.json \
    "$TAG, tools/profile_round.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py (CSVs in profiles/${TAG}_pmc/)"
cp $R/${TAG}_bench.json profiles/${TAG}_bench.json
python3 - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
out = {c: json.load(open(f"gpurun_out/cfg/{c}.json")) for c in ("c2", "c4", "c5")}
json.dump(out, open(f"profiles/{tag}_configs.json", "w"), indent=1)
lines = [l for l in open("gpurun_out/rehearse2.json") if l.startswith('{"metric"')]
open(f"profiles/{tag}_rehearse_2ranks_1gpu.json", "w").write(lines[-1])
PY
python3 tools/layer_parity_table.py gpurun_out/layer_parity_*.json > profiles/${TAG}_layer_parity.txt
echo collected
