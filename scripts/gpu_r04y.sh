#!/bin/bash
# r04 box 28: small X-stream TN blocks (one-pass reduce of their partials): 32 (in-tree) vs 16 / 64
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04y
mkdir -p $O
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  for arm in tn32 tn16 tn64; do
    lib=""; [ $arm != tn32 ] && lib="PGCN_LIB=parallel-gcn_amd/ab_$arm/libpgcn.so"
    env $lib $B --out $O/${arm}_$i.json > $O/${arm}_$i.log 2>&1 || exit $?
    summ $O/${arm}_$i.json $arm
  done
done
