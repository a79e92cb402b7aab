#!/bin/bash
# r05 late: the sparse reddit-11.6M GraphSum -- ring vs the blocked plain kernels (k_graphsum16 and
# the interleaved k_graphsum<4, 16>), one call each; then the epoch on the interleaved plain path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "blocked_gather16 or with_values" > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/gs_sparse.py 20 > $O/gs_sparse.json 2> $O/gs_sparse.err || exit $?
cat $O/gs_sparse.json
timeout -k 10 300 python3 bench.py --workload reddit-11.6M --no-extra --no-cpu-baseline > $O/b_ring.json 2> $O/b_ring.err || exit $?
timeout -k 10 300 python3 bench.py --workload reddit-11.6M --no-extra --no-cpu-baseline --knob lds_min_kb=1073741824 --knob gs16_gather=1 > $O/b_plain.json 2> $O/b_plain.err || exit $?
python3 -c "
import json
for a in ('ring','plain'):
    d=json.loads(open('$O/b_'+a+'.json').read().strip().splitlines()[-1]); print(a, d['value'], d['ms_per_step'])
"
timeout -k 10 400 python3 tools/datasets_bench.py --out $O/datasets.json > $O/datasets.log 2>&1 || exit $?
tail -3 $O/datasets.log | cut -c1-300
