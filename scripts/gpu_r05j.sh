#!/bin/bash
# r05: push-combine grid (workgroups per CU) at W = 8, solo rank epochs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05j
mkdir -p $O
for c in 2 1 4 8 2; do
  PGCN_PUSH_WG_PER_CU=$c RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 200 python3 tools/rank_epoch.py 8 > $O/rank_epoch_c$c.json 2> $O/rank_epoch_c$c.err || exit $?
  echo "cap $c: $(grep world $O/rank_epoch_c$c.err)"
done
