#!/bin/bash
# 4-layer hidden-128 reddit-114M bench (BASELINE configs[4] at one GPU) + its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python3 bench.py --hidden 128,128,128 --steps 5 --warmup 1 --no-extra > gpurun_out/bench_deep.log 2>&1; rc=$?; tail -1 gpurun_out/bench_deep.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_deep -o run -f csv -- \
    python3 bench.py --profile-only --hidden 128,128,128 --steps 3 --warmup 1 > gpurun_out/rocprof_deep.log 2>&1; rc=$?; echo rocprof rc=$rc; exit $rc
