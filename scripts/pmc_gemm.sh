#!/bin/bash
# SQ / TA counter passes over the wide-GEMM micro-benchmark (tools/gemm_wide_micro.py), one pass
# per counter group.  usage: scripts/pmc_gemm.sh <outdir-under-gpurun_out>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pmc_gemm}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run -f csv -- python3 tools/gemm_wide_micro.py \
      > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 "$OUT/$name.log"; return $rc
}
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES || exit $?
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC || exit $?
python3 tools/pmc_summary.py "$OUT" k_gemm > "$OUT/summary.txt"
cat "$OUT/summary.txt"
