#!/bin/bash
# r05: column blocks of the edge-cut rank's ring schedule (lds_blocks) at worlds 2 / 4 / 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05p
mkdir -p $O
for w in 8 4 2; do
  for nb in 0 1 2 4; do
    RANK_KNOBS=lds_blocks=$nb RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 200 python3 tools/rank_epoch.py $w > $O/w${w}_nb$nb.json 2> $O/w${w}_nb$nb.err || exit $?
    echo "lds_blocks $nb: $(grep world $O/w${w}_nb$nb.err)"
  done
done
