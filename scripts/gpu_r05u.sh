#!/bin/bash
# r05: fused wait A/B (PGCN_FUSED_WAIT 1 / 0), W = 8 and W = 4 solo rank epochs, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05u
mkdir -p $O
for i in 1 2 3; do
  for f in 1 0; do
    PGCN_FUSED_WAIT=$f RANK_STEPS=40 RANK_WARMUP=20 timeout -k 10 200 python3 tools/rank_epoch.py 8,4 > $O/fw${f}_$i.json 2> $O/fw${f}_$i.err || exit $?
    echo "fused $f: $(grep world $O/fw${f}_$i.err | tr '\n' ' ')"
  done
done
