#!/bin/bash
# r05: eval_tail on the high-priority comm stream
# peer tests (separate processes take it; loopback ranks do not), W = 8 rank epochs on / off,
# the W = 8 trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s
mkdir -p $O
ROOT=$(pwd)
timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 150 --timeout-method thread \
  tests/test_gpu_peer_procs.py tests/test_gpu_multirank.py > $O/pytest_peer.log 2>&1
rc=$?; echo "peer tests rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_peer.log | head -30; tail -2 $O/pytest_peer.log
[ $rc -eq 0 ] || exit $rc
for t in 1 0 1 0; do
  RANK_KNOBS=eval_tail=$t RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 200 python3 tools/rank_epoch.py 8 > $O/w8_tail$t.json 2> $O/w8_tail$t.err || exit $?
  echo "eval_tail $t: $(grep world $O/w8_tail$t.err)"
done
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rank8 -o run -f csv -- \
    python3 tools/rank_epoch.py 8 0 16 > $O/prof_rank8.log 2>&1; rc=$?; echo "rank8 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(dirname $(find $O/prof_rank8 -name run_kernel_trace.csv | head -1))
python3 tools/epoch_breakdown.py $T > $O/rank8_breakdown.txt 2>&1; head -5 $O/rank8_breakdown.txt
