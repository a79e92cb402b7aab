#!/bin/bash
# Kernel trace of one edge-cut rank's epoch at world W on one GPU (timing-only communicator,
# tools/rank_epoch.py).  usage: scripts/prof_rank.sh <world> [hidden]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
W=${1:-8}; H=${2:-16}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_rank$W" -o run -f csv -- \
    python3 tools/rank_epoch.py "$W" 0 "$H" > "gpurun_out/prof_rank$W.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 "gpurun_out/prof_rank$W.log"; exit $rc; }
