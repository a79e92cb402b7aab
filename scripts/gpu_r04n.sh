#!/bin/bash
# r04 box 14: ring GraphSum rowsets in pairs with both blocks' table reads in flight
# (PGCN_RING_PIPE=1 build, ab_pipe): GraphSum GPU tests on that build, GraphSum alone and the
# epoch against the in-tree build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04n
mkdir -p $O
PGCN_LIB=parallel-gcn_amd/ab_pipe/libpgcn.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "graphsum or lds" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for arm in tree pipe; do
  env=""; [ $arm = pipe ] && env="PGCN_LIB=parallel-gcn_amd/ab_pipe/libpgcn.so"
  env $env timeout -k 10 200 python3 tools/gs_call.py 30 > $O/gs_$arm.json 2> $O/gs_$arm.err || exit $?
  echo "gs $arm $(cat $O/gs_$arm.json)"
done
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1))"; }
for i in 1 2 3; do
  for arm in tree pipe; do
    env=""; [ $arm = pipe ] && env="PGCN_LIB=parallel-gcn_amd/ab_pipe/libpgcn.so"
    env $env timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-extra \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
