#!/bin/bash
# r04 box 25: plain GraphSum item length with workgroup items (gs_split 3): 8 (default) vs 4 / 2
# group iterations per item (shorter items: more rows summed by whole workgroups)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04w
mkdir -p $O
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  for it in 8 4 2; do
    $B --set gs_item_iters=$it --out $O/i${it}_$i.json > $O/i${it}_$i.log 2>&1 || exit $?
    summ $O/i${it}_$i.json i$it
  done
done
