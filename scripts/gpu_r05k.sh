#!/bin/bash
# r05: push combine grid x sc1 ring partials at W = 8 (solo rank epochs), then the trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05k
mkdir -p $O
ROOT=$(pwd)
for arm in "1 0" "1 1" "2 1" "4 1" "1 0" "1 1"; do
  set -- $arm
  PGCN_PUSH_WG_PER_CU=$1 PGCN_PART_SC1=$2 RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 200 python3 tools/rank_epoch.py 8 > $O/re_$1_$2.json 2> $O/re_$1_$2.err || exit $?
  echo "cap $1 sc1 $2: $(grep world $O/re_$1_$2.err)"
done
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PGCN_PUSH_WG_PER_CU=1 PGCN_PART_SC1=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rank8 -o run -f csv -- \
    python3 tools/rank_epoch.py 8 0 16 > $O/prof_rank8.log 2>&1; rc=$?; echo "rank8 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(dirname $(find $O/prof_rank8 -name run_kernel_trace.csv | head -1))
python3 tools/epoch_breakdown.py $T > $O/rank8_breakdown.txt 2>&1; head -12 $O/rank8_breakdown.txt
