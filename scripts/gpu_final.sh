#!/bin/bash
# Round-end evidence on one box: smoke, GPU tests, bench (CPU leg on), kernel trace, PMC
# FETCH/WRITE passes (separate runs) -> per-call GraphSum traffic, the 4-layer hidden-128 bench
# + trace, the small datasets.  Stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_round.sh || exit $?
PASSES="fetch write" bash scripts/profile.sh prof_pmc || exit $?
python3 tools/traffic.py gpurun_out/prof_pmc > gpurun_out/traffic.json || exit $?
cat gpurun_out/traffic.json
bash scripts/gpu_deep.sh || exit $?
timeout -k 10 400 python3 tools/datasets_bench.py --epochs 300 --graph 0 --out gpurun_out/datasets.json > gpurun_out/datasets.log 2>&1; echo datasets rc=$?
