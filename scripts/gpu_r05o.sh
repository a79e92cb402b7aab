#!/bin/bash
# r05: GraphSum bulk outputs (ring partials, combine output, next tables) stored past the L2
# (PGCN_STORE_SC1 build, ab_sc1): GraphSum tests on that build, then the epoch A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05o
mkdir -p $O
PGCN_LIB=parallel-gcn_amd/ab_sc1/libpgcn.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q -k "graphsum or epilogue or bit_identical" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];m=d['mfma'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1), 'xs+gemm', round(m['ms_per_epoch']*1e3,1))"; }
for i in 1 2 3; do
  for arm in base sc1; do
    env=""; [ $arm = sc1 ] && env="PGCN_LIB=parallel-gcn_amd/ab_sc1/libpgcn.so"
    env $env timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
