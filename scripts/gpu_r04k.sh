#!/bin/bash
# r04 box 11: full GPU suite; the sparse-X SpMM kernels (csr: the next batch's loads with this
# batch's gathers, the keep test at use; csc: value / mask / G in one round trip, 1,024-entry
# chunks for long columns) against HEAD's build on the small datasets, twice each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for arm in head new; do
    env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
    env $env timeout -k 10 300 python3 tools/datasets_bench.py --epochs 300 --graph 0 --no-cpu --out $O/ds_${arm}_$i.json > $O/ds_${arm}_$i.log 2>&1 || exit $?
    python3 -c "
import json; d=json.load(open('$O/ds_${arm}_$i.json'))
print('$arm', ' '.join(f'{k} {v.get(\"eager_async_epochs_s\",0):.0f}' for k,v in d.items() if isinstance(v, dict)))"
  done
done
