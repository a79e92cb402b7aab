#!/bin/bash
# r05 evidence box B: rank epochs at HEAD (worlds 1..8; W = 8 column blocks 2 / 4 / 8), the
# traced headline (event vs rocprof GraphSum fraction, breakdown), PMC FETCH / WRITE passes of
# the headline and of the 4-layer hidden-128 model, the reddit-11.6M and 4-layer bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUTDIR:-r05n}
mkdir -p $O
ROOT=$(pwd)
RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 400 python3 tools/rank_epoch.py 1,2,4,8 > $O/rank_epoch.json 2> $O/rank_epoch.err; rc=$?
echo "rank_epoch rc=$rc"; grep world $O/rank_epoch.err; [ $rc -eq 0 ] || exit $rc
for nb in 2 8; do
  RANK_KNOBS=lds_blocks=$nb RANK_STEPS=30 RANK_WARMUP=20 timeout -k 10 200 python3 tools/rank_epoch.py 8 > $O/rank8_nb$nb.json 2> $O/rank8_nb$nb.err || exit $?
  echo "lds_blocks $nb: $(grep world $O/rank8_nb$nb.err)"
done
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --no-cpu-baseline --no-extra > $O/trace_bench.json 2> $O/trace.log; rc=$?
echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/gs_fraction.py $O/trace $O/trace_bench.json > $O/gs_fraction.json; cat $O/gs_fraction.json
python3 tools/epoch_breakdown.py $O/trace > $O/breakdown.txt 2>&1; head -14 $O/breakdown.txt
PASSES="trace fetch write" bash scripts/profile.sh ${OUTDIR:-r05n}/pmc || exit $?
PASSES="fetch write" bash scripts/profile.sh ${OUTDIR:-r05n}/pmc4 --hidden 128,128,128 || exit $?
timeout -k 10 600 python3 bench.py --workload reddit-11.6M > $O/bench_11.6M.json 2> $O/bench_11.6M.err; echo "11.6M rc=$?"; cut -c1-300 $O/bench_11.6M.json
timeout -k 10 900 python3 bench.py --hidden 128,128,128 --steps 20 --warmup 5 > $O/bench_4layer.json 2> $O/bench_4layer.err; echo "4layer rc=$?"; cut -c1-300 $O/bench_4layer.json
