#!/bin/bash
# PMC counter passes over a short bench.py run (one rocprofv3 run per pass;
# counters only, no tracing domains).  Output: gpurun_out/pmc/<pass>/...csv,
# summarised by tools/pmc_summary.py.
#   tools/pmc.sh [bench.py args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc
mkdir -p "$OUT"
BENCH=(python3 "$PWD/bench.py" --steps 2 --warmup 1 --profile-steps 1 --cpu-sample 0 "$@")
PASSES=(
  "cyc:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
  "ins:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM"
  "lds:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"
  "fetch:FETCH_SIZE"
  "write:WRITE_SIZE"
  "tcc:TCC_HIT_sum TCC_MISS_sum"
)
for p in "${PASSES[@]}"; do
  name=${p%%:*}; ctr=${p#*:}
  echo "[$(date +%T)] pmc pass $name: $ctr"
  ( cd /tmp && timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o run -- "${BENCH[@]}" ) > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] pass $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" | tee "$OUT/summary.txt"
