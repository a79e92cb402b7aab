#!/bin/bash
# rocprofv3 PMC passes over the GraphSum micro-benchmark (tools/gs_micro.py <config>), one
# counter group per pass, no trace domains beside --pmc.
# usage: scripts/profile_gs.sh <outdir-under-gpurun_out> [config=lds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gsprof}
CFG=${2:-lds}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run -f csv -- python3 tools/gs_micro.py "$CFG" \
      > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -20 "$OUT/$name.log"; return $rc
}
run trace --kernel-trace --stats || exit $?
run lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES || exit $?
run sq --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VALU || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
