#!/bin/bash
# r05: the W1.grad csc pass's workgroups in descending column length -- sparse-X tests, then the
# small-graph A/B against the previous library (ab_prev, built from HEAD~)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_engine.py -k "csc or spmm or cora or citeseer or pubmed or sparse" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in new prev; do
    env=""; [ $arm = prev ] && env="PGCN_LIB=parallel-gcn_amd/ab_prev/libpgcn.so"
    env $env timeout -k 10 300 python3 tools/datasets_bench.py --no-cpu --out $O/ds_${arm}_$i.json > $O/ds_${arm}_$i.log 2>&1 || exit $?
    python3 -c "import json;d=json.load(open('$O/ds_${arm}_$i.json'));print('$arm', {k:round(v['eager_async_epochs_s']) for k,v in d.items() if isinstance(v,dict) and 'eager_async_epochs_s' in v})"
  done
done
