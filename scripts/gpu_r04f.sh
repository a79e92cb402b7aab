#!/bin/bash
# r04 box 6: full GPU suite; A/B against HEAD's build (ab_head) of the GraphSum tails loading
# their inputs up front (combine / finish / plain kernels' epilogue loads, the ring's row
# words); small graphs both ways; stamped traffic passes of the changed ring sources.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1))"; }
for i in 1 2 3; do
  for arm in head new; do
    env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
    env $env timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
for arm in head new; do
  env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
  env $env timeout -k 10 400 python3 tools/datasets_bench.py --epochs 300 --graph 0 --out $O/datasets_$arm.json > $O/datasets_$arm.log 2>&1
  echo "datasets $arm rc=$?"; python3 -c "
import json; d=json.load(open('$O/datasets_$arm.json'))
for k,v in d.items():
    if isinstance(v, dict): print('$arm', k, round(v.get('eager_async_epochs_s',0),1), round(v.get('eager_frac_of_launch_floor',0),3))"
done
bash scripts/gpu_traffic.sh r04f_traffic
