#!/bin/bash
# r04 box 9: the bench lines of HEAD (headline with CPU leg + parity, reddit-11.6M, 4-layer,
# small datasets, the headline's rocprofv3 trace) and the edge-cut rank epochs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_lines.sh || exit $?
timeout -k 10 300 python3 tools/rank_epoch.py 1,2,4,8 0 16 > gpurun_out/rank_epoch_i.json 2> gpurun_out/rank_epoch_i.err
echo "rank_epoch rc=$?"; cat gpurun_out/rank_epoch_i.json
