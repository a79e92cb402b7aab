#!/bin/bash
# rocprofv3 passes over the bench workload: kernel trace + stats, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE never share a pass, MI355X_MICROARCH.md).
# PMC passes carry no sys/runtime/hip traces.
# usage: scripts/profile.sh <outdir-under-gpurun_out> [bench args...]
# env PASSES="trace fetch write l2" selects passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-prof}; shift || true
ARGS="--profile-only --steps 3 --warmup 1 $*"
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" -d "$OUT/$name" -o run -f csv -- python3 bench.py $ARGS \
      > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -20 "$OUT/$name.log"; return $rc
}
for p in ${PASSES:-trace fetch write}; do
  case $p in
    trace) run trace --kernel-trace --stats || exit $? ;;
    fetch) run fetch --pmc FETCH_SIZE || exit $? ;;
    write) run write --pmc WRITE_SIZE || exit $? ;;
    l2) run l2 --pmc TCC_HIT_sum TCC_MISS_sum || exit $? ;;
  esac
done
