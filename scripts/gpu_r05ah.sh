#!/bin/bash
# r05 late: the X-stream ring kernels read the flat dropout bitmap (second box: the A/B after
# r05ag's suite and parity line) -- the X-stream kernel tests, a same-box A/B against HEAD
# (ab_prev), three pairs, and a traced breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -k "xstream or gemm" -v -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in new prev; do
    env=""; [ $arm = prev ] && env="PGCN_LIB=parallel-gcn_amd/ab_prev/libpgcn.so"
    env $env timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra > $O/b_${arm}_$i.json 2> $O/b_${arm}_$i.err || exit $?
    python3 -c "import json;d=json.loads(open('$O/b_${arm}_$i.json').read().strip().splitlines()[-1]);print('$arm', round(d['value'],1), d['ms_per_step'])"
  done
done
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --no-cpu-baseline --no-extra > $O/trace_bench.json 2> $O/trace.log || exit $?
python3 tools/epoch_breakdown.py $O/trace > $O/breakdown.txt 2>&1; head -16 $O/breakdown.txt
