#!/bin/bash
# r05 closing box B: traced headline (event vs rocprof fraction, breakdown), PMC FETCH / WRITE
# passes at HEAD, solo rank epochs and the W = 8 trace, reddit-11.6M and 4-layer lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05final
mkdir -p $O
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --no-cpu-baseline --no-extra > $O/trace_bench.json 2> $O/trace.log; rc=$?
echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/gs_fraction.py $O/trace $O/trace_bench.json > $O/gs_fraction.json; cat $O/gs_fraction.json
python3 tools/epoch_breakdown.py $O/trace > $O/breakdown.txt 2>&1; head -3 $O/breakdown.txt
PASSES="fetch write" bash scripts/profile.sh r05final/pmc || exit $?
RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 400 python3 tools/rank_epoch.py 1,2,4,8 > $O/rank_epoch.json 2> $O/rank_epoch.err; rc=$?
echo "rank_epoch rc=$rc"; grep world $O/rank_epoch.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rank8 -o run -f csv -- \
    python3 tools/rank_epoch.py 8 0 16 > $O/prof_rank8.log 2>&1; rc=$?; echo "rank8 trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(dirname $(find $O/prof_rank8 -name run_kernel_trace.csv | head -1))
python3 tools/epoch_breakdown.py $T > $O/rank8_breakdown.txt 2>&1; head -3 $O/rank8_breakdown.txt
timeout -k 10 600 python3 bench.py --workload reddit-11.6M > $O/bench_11.6M.json 2> $O/bench_11.6M.err; echo "11.6M rc=$?"; cut -c1-200 $O/bench_11.6M.json
timeout -k 10 900 python3 bench.py --hidden 128,128,128 --steps 20 --warmup 5 > $O/bench_4layer.json 2> $O/bench_4layer.err; echo "4layer rc=$?"; cut -c1-200 $O/bench_4layer.json
timeout -k 10 600 python3 bench.py > $O/bench_head.json 2> $O/bench_head.err; echo "bench (logits parity) rc=$?"; python3 -c "import json;d=json.load(open('$O/bench_head.json'));print(d['value'], d['parity'].get('logits'), d['parity']['pass'])"
