#!/bin/bash
# HBM traffic of the d = 128 GraphSum (reddit-114M bench graph, tools/gs_call.py: one warm-up
# call + 5 timed), FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes; per-call bytes by
# tools/traffic.py over the last 5 calls' 8 ring passes (usage: scripts/pmc_wide.sh [outdir])
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pmc_wide}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/$c" -o run -f csv -- python3 tools/gs_call.py 5 128 \
      > "$OUT/$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$c.log"; exit $rc; }
done
python3 tools/traffic.py "$OUT" 40 > "$OUT/traffic_passes.json" && cat "$OUT/traffic_passes.json"
grep -h ms_per_call "$OUT"/FETCH_SIZE.log | tail -1
