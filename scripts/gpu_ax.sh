#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ax_build.py > gpurun_out/ax_build.json 2> gpurun_out/ax_build.err; echo "rc=$?"; cat gpurun_out/ax_build.json
