#!/bin/bash
# Full round check on one GPU box: smoke, GPU tests, bench (with the CPU reference leg),
# rocprofv3 kernel trace of the bench.  Stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -5 "gpurun_out/$name.log"; return $rc
}
[ -n "${SKIP_TESTS:-}" ] || step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_gpu 1000 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} || exit $?
fi
step bench 600 python3 bench.py ${BENCH_ARGS:-} || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run -f csv -- \
    python3 bench.py --profile-only --steps 5 --warmup 1 || exit $?
