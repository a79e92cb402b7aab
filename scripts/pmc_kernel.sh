#!/bin/bash
# SQ counter passes (one per group) over the bench workload, restricted to kernels matching a
# regex, then per-kernel averages.  usage: scripts/pmc_kernel.sh <tag> <kernel-regex> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmc}; RX=${2:-.}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" -d "$OUT/$name" -o run -f csv -- \
      python3 bench.py --profile-only --steps 3 --warmup 1 "${BARGS[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 "$OUT/$name.log"; return $rc
}
BARGS=("$@")
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS || exit $?
pass sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM || exit $?
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
