#!/bin/bash
# r04 box 26: item length by shape (gs_item_iters 0, default) -- GPU tests of the GraphSum and
# engine paths, then the datasets A/B against 8 and 2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  for it in 0 8 2; do
    $B --set gs_item_iters=$it --out $O/i${it}_$i.json > $O/i${it}_$i.log 2>&1 || exit $?
    summ $O/i${it}_$i.json i$it
  done
done
timeout -k 10 400 python3 tools/datasets_bench.py --out $O/datasets.json > $O/datasets.log 2>&1; echo "datasets rc=$?"; tail -3 $O/datasets.log | cut -c1-120
