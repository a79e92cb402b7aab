#!/bin/bash
# The other bench lines (reddit-11.6M, 4-layer hidden 128, small datasets), then the d = 128
# GraphSum PMC traffic (scripts/pmc_wide.sh).  Stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; return $rc
}
step bench_116 600 python3 bench.py --workload reddit-11.6M --no-extra || exit $?
step bench_deep 500 python3 bench.py --hidden 128,128,128 --steps 5 --warmup 1 --no-extra || exit $?
step datasets 400 python3 tools/datasets_bench.py --out gpurun_out/datasets.json || exit $?
bash scripts/pmc_wide.sh pmc_wide
