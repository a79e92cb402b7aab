#!/bin/bash
# r05: eval_ax (Â X precomputed at build, charged over 100 epochs) against train_ahead over X
# (eval_ax 0), interleaved; the W = 8 rank epoch with 2 column blocks by default; multirank tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05q
mkdir -p $O
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1))"; }
for i in 1 2; do
  for arm in ax ahead; do
    k=""; [ $arm = ahead ] && k="--knob eval_ax=0"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra $k > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 400 python3 tools/rank_epoch.py 1,2,4,8 > $O/rank_epoch.json 2> $O/rank_epoch.err; rc=$?
echo "rank_epoch rc=$rc"; grep world $O/rank_epoch.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 150 --timeout-method thread \
  tests/test_gpu_peer_procs.py tests/test_gpu_multirank.py > $O/pytest_peer.log 2>&1
rc=$?; echo "peer tests rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_peer.log | head -30; tail -2 $O/pytest_peer.log; exit $rc
