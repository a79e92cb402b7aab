#!/bin/bash
# r04 box 17: small-graph launch and latency cuts -- GPU tests of the in-kernel split-row
# combine, co-drawn masks, Matmul backward tails and the U-entry csc backward; then the
# datasets A/B: "old" = U 1 build (ab_u1) with every new knob off, "new" = defaults (item
# length 8 iterations), and the item lengths 4 / 16
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q \
    -k "split_rows or co_draw or graphsum_vs_oracle or fused_epilogue or cora or spmm or dropout" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  PGCN_LIB=parallel-gcn_amd/ab_u1/libpgcn.so $B --set gs_split=0 --set fuse_epilogue=7 --set co_draw=0 --set gs_item_iters=32 --out $O/old_$i.json > $O/old_$i.log 2>&1 || exit $?
  summ $O/old_$i.json old
  $B --out $O/new_$i.json > $O/new_$i.log 2>&1 || exit $?
  summ $O/new_$i.json new8
  $B --set gs_item_iters=4 --out $O/it4_$i.json > $O/it4_$i.log 2>&1 || exit $?
  summ $O/it4_$i.json it4
  $B --set gs_item_iters=16 --out $O/it16_$i.json > $O/it16_$i.log 2>&1 || exit $?
  summ $O/it16_$i.json it16
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o cora -- python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 500 --only cora > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats_cora.csv
