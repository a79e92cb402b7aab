#!/bin/bash
# r04 box 10: full GPU suite; A/B against HEAD's build (ab_head) of the ring GraphSum's visit
# hand-offs in one LDS round trip (done count + next visit's word + count); GraphSum alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for arm in head new; do
  env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
  env $env timeout -k 10 200 python3 tools/gs_call.py 30 > $O/gs_$arm.json 2> $O/gs_$arm.err || exit $?
  echo "gs $arm $(cat $O/gs_$arm.json)"
done
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1))"; }
for i in 1 2 3; do
  for arm in head new; do
    env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
    env $env timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
