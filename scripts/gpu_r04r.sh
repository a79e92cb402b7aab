#!/bin/bash
# r04 box 18: workgroup items for the small graphs' hub rows (gs_split 3) -- GPU tests, then
# the datasets A/B: "old" = U 1 build (ab_u1) with the new knobs off; defaults (gs_split 3,
# 8-iteration items); gs_split 3 at 16 / 32; gs_split 1 at 16; then a cora kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q \
    -k "split_rows or co_draw or graphsum or fused_epilogue or cora or spmm or dropout or epoch_lines or epoch1" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000"
summ() { python3 -c "import json;d=json.load(open('$1'));print('$2', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"; }
for i in 1 2 3; do
  PGCN_LIB=parallel-gcn_amd/ab_u1/libpgcn.so $B --set gs_split=0 --set fuse_epilogue=7 --set co_draw=0 --set gs_item_iters=32 --out $O/old_$i.json > $O/old_$i.log 2>&1 || exit $?
  summ $O/old_$i.json old
  $B --out $O/s3i8_$i.json > $O/s3i8_$i.log 2>&1 || exit $?
  summ $O/s3i8_$i.json s3i8
  $B --set gs_item_iters=16 --out $O/s3i16_$i.json > $O/s3i16_$i.log 2>&1 || exit $?
  summ $O/s3i16_$i.json s3i16
  $B --set gs_item_iters=32 --out $O/s3i32_$i.json > $O/s3i32_$i.log 2>&1 || exit $?
  summ $O/s3i32_$i.json s3i32
  $B --set gs_split=1 --set gs_item_iters=16 --out $O/s1i16_$i.json > $O/s1i16_$i.log 2>&1 || exit $?
  summ $O/s1i16_$i.json s1i16
done
for d in cora pubmed_synth; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$d -o run -f csv -- python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 500 --only $d > $O/prof_$d.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', round(d['value'],1), d['roofline']['frac'])"
