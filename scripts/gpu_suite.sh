#!/bin/bash
# One GPU-box check: smoke, the whole GPU test suite, a short bench line.  Stops at the first
# failing step.  usage: scripts/gpu_suite.sh <tag> [pytest args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-suite}; shift || true
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -4 "gpurun_out/${TAG}_$name.log"; return $rc
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest 1000 python3 -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread "$@" || exit $?
[ -n "${SKIP_BENCH:-}" ] || step bench 600 python3 bench.py --no-cpu-baseline --no-extra || exit $?
