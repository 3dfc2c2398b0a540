#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over build/pmc_calib (one counter
# per rocprofv3 run), then tools/pmc_calib.py's counted / moved table.
#   tools/pmc_calib.sh            (GPU box, repo root; build/pmc_calib prebuilt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
BIN=$PWD/build/pmc_calib
OUT=$PWD/gpurun_out/pmc_calib; mkdir -p "$OUT"
( cd /tmp && timeout -k 10 60 "$BIN" ) > "$OUT/plain.log" 2>&1 || { cat "$OUT/plain.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$OUT/$c" -o calib -- "$BIN" ) > "$OUT/$c.log" 2>&1
  rc=$?
  echo "$c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/$c.log"; exit $rc; }
done
python3 tools/pmc_calib.py "$OUT"
