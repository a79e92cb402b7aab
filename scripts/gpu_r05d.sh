#!/bin/bash
# r05: the edge-cut rank epoch on the peer exchange's kernels (solo form) at worlds 1/2/4/8,
# the W = 8 rank's kernel trace, and the default bench line with its rocprof summary
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05d
mkdir -p $O
ROOT=$(pwd)
timeout -k 10 400 python3 tools/rank_epoch.py 1,2,4,8 > $O/rank_epoch.json 2> $O/rank_epoch.err; rc=$?
echo "rank_epoch rc=$rc"; cat $O/rank_epoch.err | grep world; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rank8 -o run -f csv -- \
    python3 tools/rank_epoch.py 8 0 16 > $O/prof_rank8.log 2>&1; rc=$?; echo "rank8 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(dirname $(find $O/prof_rank8 -name run_kernel_trace.csv | head -1))
python3 tools/epoch_breakdown.py $T > $O/rank8_breakdown.txt 2>&1; cat $O/rank8_breakdown.txt | head -30
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run -f csv -- \
    python3 bench.py --profile-only --steps 20 --warmup 5 > $O/prof_bench.log 2>&1; rc=$?; echo "bench trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(dirname $(find $O/prof_bench -name run_kernel_trace.csv | head -1))
python3 tools/epoch_breakdown.py $T > $O/bench_breakdown.txt 2>&1; cat $O/bench_breakdown.txt | head -30
