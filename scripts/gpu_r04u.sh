#!/bin/bash
# r04 box 22: csc prefetch in the 1024-thread form only -- spmm bit-exact tests, A/B against the
# U 1 kernel (ab_prev), then the small datasets with their CPU legs (closing numbers)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q -k "spmm or epoch1 or epoch_lines" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  PGCN_LIB=parallel-gcn_amd/ab_prev/libpgcn.so $B --out $O/prev_$i.json > $O/prev_$i.log 2>&1 || exit $?
  summ $O/prev_$i.json prev
  $B --out $O/new_$i.json > $O/new_$i.log 2>&1 || exit $?
  summ $O/new_$i.json new
done
timeout -k 10 400 python3 tools/datasets_bench.py --out $O/datasets.json > $O/datasets.log 2>&1; echo "datasets rc=$?"; tail -3 $O/datasets.log | cut -c1-200
