#!/bin/bash
# r04 box 16: small-graph launch cuts -- in-kernel combine of split GraphSum rows (gs_split 1)
# and the Dropout + ReLU backward in the Matmul input-grad product (fuse_epilogue bit 8):
# their GPU tests, then datasets_bench A/B against both off (gs_split 0, fuse_epilogue 7)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q \
    -k "split_rows_in_kernel or graphsum_vs_oracle or fused_epilogue or cora" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000 --set gs_split=0 --set fuse_epilogue=7 --out $O/old_$i.json > $O/old_$i.log 2>&1 || exit $?
  timeout -k 10 300 python3 tools/datasets_bench.py --graph 0 --no-cpu --epochs 2000 --out $O/new_$i.json > $O/new_$i.log 2>&1 || exit $?
  for arm in old new; do
    python3 -c "import json;d=json.load(open('$O/${arm}_$i.json'));print('$arm', *[(k, round(d[k]['eager_async_epochs_s']), d[k]['launches_per_epoch']) for k in ('cora','citeseer','pubmed_synth')])"
  done
done
