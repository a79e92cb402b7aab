#!/bin/bash
# r04 box 23: eval's sparse product also computing the next training forward's (sparse_dual):
# the small-graph engine tests, then the datasets A/B sparse_dual 0 vs 1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  $B --set sparse_dual=0 --out $O/off_$i.json > $O/off_$i.log 2>&1 || exit $?
  summ $O/off_$i.json off
  $B --out $O/on_$i.json > $O/on_$i.log 2>&1 || exit $?
  summ $O/on_$i.json on
done
