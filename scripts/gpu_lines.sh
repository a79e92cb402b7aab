#!/bin/bash
# Bench lines of one build on one box: the headline (reddit-114M 2-layer, with the CPU reference
# leg and parity), the report-comparable reddit-11.6M workload (with its CPU leg), the 4-layer
# hidden-128 line, the small datasets; then the rocprofv3 kernel trace of the headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400; return $rc
}
step bench 600 python3 bench.py || exit $?
step bench_116 600 python3 bench.py --workload reddit-11.6M --no-extra || exit $?
step bench_deep 500 python3 bench.py --hidden 128,128,128 --steps 5 --warmup 1 --no-extra || exit $?
step datasets 400 python3 tools/datasets_bench.py --out gpurun_out/datasets.json || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run -f csv -- \
    python3 bench.py --profile-only --steps 5 --warmup 1 || exit $?
