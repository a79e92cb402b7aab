#!/bin/bash
# r05: the W = 8 solo rank epoch under the profiler (cached sc0 sc1 pushes), rank epochs settled
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05g
mkdir -p $O
ROOT=$(pwd)
RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 400 python3 tools/rank_epoch.py 1,2,4,8 > $O/rank_epoch.json 2> $O/rank_epoch.err; rc=$?
echo "rank_epoch rc=$rc"; grep world $O/rank_epoch.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rank8 -o run -f csv -- \
    python3 tools/rank_epoch.py 8 0 16 > $O/prof_rank8.log 2>&1; rc=$?; echo "rank8 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(dirname $(find $O/prof_rank8 -name run_kernel_trace.csv | head -1))
python3 tools/epoch_breakdown.py $T > $O/rank8_breakdown.txt 2>&1; head -40 $O/rank8_breakdown.txt
