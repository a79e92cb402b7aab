#!/bin/bash
# r05: the next input mask on the side stream (LDS-free k_dropout_mask_side beside the ring
# GraphSums, knob mask_side) -- its bit-identity tests, the peer tests with cached slots, then
# the epoch A/B (mask_side 0 / 1 / 2, interleaved)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -m gpu -v -x --timeout 150 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_engine.py -k "mask_side or train_ahead or dropout or gemm_xstream" > $O/pytest_mask.log 2>&1
rc=$?; echo "mask tests rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_mask.log | head -20; tail -2 $O/pytest_mask.log
[ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];m=d['mfma'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1), 'xs+gemm', round(m['ms_per_epoch']*1e3,1))"; }
for i in 1 2 3; do
  for arm in 0 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra --knob mask_side=$arm \
        > $O/ab_side${arm}_$i.json 2> $O/ab_side${arm}_$i.err || exit $?
    summ $O/ab_side${arm}_$i.json side$arm
  done
done
timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 150 --timeout-method thread \
  tests/test_gpu_peer_procs.py tests/test_gpu_multirank.py > $O/pytest_peer.log 2>&1
rc=$?; echo "peer tests rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_peer.log | head -30; tail -2 $O/pytest_peer.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/rank_epoch.py 1,2,4,8 > $O/rank_epoch.json 2> $O/rank_epoch.err; rc=$?
echo "rank_epoch rc=$rc"; grep world $O/rank_epoch.err; exit $rc
