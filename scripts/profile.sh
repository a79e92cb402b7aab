#!/bin/bash
# rocprofv3 passes over the bench workload (kernel trace + separate PMC passes, as the
# MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE never share a pass).
# usage: scripts/profile.sh <outdir-under-gpurun_out> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-prof}; shift || true
ARGS="--profile-only --steps 3 --warmup 1 $*"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" -d "$OUT/$name" -o run -f csv -- python3 bench.py $ARGS \
      > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
run trace --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run l2 --pmc TCC_HIT_sum TCC_MISS_sum || exit $?
run sq --pmc SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES || exit $?
