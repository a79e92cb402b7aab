#!/bin/bash
# r04 box 20: csc backward with column-major LDS products and its add chain's reads a batch
# ahead (in-tree) vs the previous commit's U 1 kernel (ab_prev): spmm bit-exact tests, the
# datasets A/B, a cora kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "spmm" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  PGCN_LIB=parallel-gcn_amd/ab_prev/libpgcn.so $B --out $O/prev_$i.json > $O/prev_$i.log 2>&1 || exit $?
  summ $O/prev_$i.json prev
  $B --out $O/new_$i.json > $O/new_$i.log 2>&1 || exit $?
  summ $O/new_$i.json new
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_cora -o run -f csv -- python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 500 --only cora > $O/prof_cora.log 2>&1 || exit $?
