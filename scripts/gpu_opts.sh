#!/bin/bash
# GraphSum option sweep, then the GPU tests and a short bench (stops at the first GPU fault,
# abort or timeout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python3 tools/gs_opts.py ${GS_OPTS:-} > gpurun_out/gs_opts.json 2> gpurun_out/gs_opts.err
rc=$?; echo "gs_opts rc=$rc"; cat gpurun_out/gs_opts.json; tail -5 gpurun_out/gs_opts.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
