#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-nothing_matches}" > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for i in 1 2; do
 for v in new old; do
  if [ $v = old ]; then export PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so; else unset PGCN_LIB; fi
  timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/ab_${v}_$i.json 2> gpurun_out/ab_${v}_$i.err || { echo bench fail $v; tail -5 gpurun_out/ab_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${v}_$i.json')); print('$v', round(d['value'],1), round(d['roofline']['avg_call_ms'],4))"
 done
done
unset PGCN_LIB
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o run -f csv -- python3 bench.py --profile-only --steps 5 --warmup 1 > gpurun_out/prof_ab.log 2>&1; echo prof rc=$?
