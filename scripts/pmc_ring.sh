#!/bin/bash
# SQ counter passes over the ring GraphSum (tools/gs_call.py: d = 16 calls on reddit-114M), one
# pass per counter group.  usage: scripts/pmc_ring.sh <outdir-under-gpurun_out> [calls]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pmc_ring}; CFG=${2:-5}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run -f csv -- python3 tools/gs_call.py $CFG \
      > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 "$OUT/$name.log"; return $rc
}
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS || exit $?
pass sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM || exit $?
python3 tools/pmc_summary.py "$OUT" k_graphsum_ring > "$OUT/summary.txt"
cat "$OUT/summary.txt"
