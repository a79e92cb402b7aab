#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gs_sparse.py 20 > gpurun_out/gs_sparse.json 2> gpurun_out/gs_sparse.err; echo "rc=$?"; cat gpurun_out/gs_sparse.json; tail -3 gpurun_out/gs_sparse.err
