#!/bin/bash
# r04 final box: full GPU suite; the bench lines (headline with CPU leg + parity, reddit-11.6M,
# 4-layer, small datasets, headline rocprofv3 trace); the event vs rocprof GraphSum fraction
# from one traced bench run; the edge-cut rank epochs; smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04final
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.log
bash scripts/gpu_lines.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/trace_bench.json 2> $O/trace.log
echo "trace rc=$?"
python3 tools/gs_fraction.py $O/trace $O/trace_bench.json > $O/gs_fraction.json; cat $O/gs_fraction.json
python3 tools/epoch_breakdown.py $O/trace > $O/breakdown.txt 2>&1; head -14 $O/breakdown.txt
timeout -k 10 300 python3 tools/rank_epoch.py 1,2,4,8 0 16 > $O/rank_epoch.json 2> $O/rank_epoch.err
echo "rank_epoch rc=$?"; cat $O/rank_epoch.json
