#!/bin/bash
# r05: the receiver's wait fused into the push launch (separate processes / solo): peer tests,
# rank epochs, the W = 8 trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05t
mkdir -p $O
ROOT=$(pwd)
timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 150 --timeout-method thread \
  tests/test_gpu_peer_procs.py tests/test_gpu_multirank.py > $O/pytest_peer.log 2>&1
rc=$?; echo "peer tests rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_peer.log | head -30; tail -2 $O/pytest_peer.log
[ $rc -eq 0 ] || exit $rc
RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 400 python3 tools/rank_epoch.py 1,2,4,8 > $O/rank_epoch.json 2> $O/rank_epoch.err; rc=$?
echo "rank_epoch rc=$rc"; grep world $O/rank_epoch.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rank8 -o run -f csv -- \
    python3 tools/rank_epoch.py 8 0 16 > $O/prof_rank8.log 2>&1; rc=$?; echo "rank8 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(dirname $(find $O/prof_rank8 -name run_kernel_trace.csv | head -1))
python3 tools/epoch_breakdown.py $T > $O/rank8_breakdown.txt 2>&1; head -20 $O/rank8_breakdown.txt
