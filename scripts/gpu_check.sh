#!/bin/bash
# One GPU-box session: GPU tests, then a short bench. Stops at the first GPU fault / abort /
# timeout (exit >= 124 or a signal), continues past ordinary test failures (exit 1).
# usage: scripts/gpu_check.sh [pytest-args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -x "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -20 gpurun_out/bench.err
exit $rc
