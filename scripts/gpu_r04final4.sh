#!/bin/bash
# r04 closing box (after the small-graph work and the sparse dual forward): full GPU suite, smoke(), the default bench.py
# line (100 epochs after 20 warmup, CPU leg + parity), the small datasets with their CPU legs,
# the traced headline (event vs rocprof GraphSum fraction, epoch breakdown)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04final4
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err; echo "bench rc=$?"; cut -c1-300 $O/bench.json
timeout -k 10 400 python3 tools/datasets_bench.py --out $O/datasets.json > $O/datasets.log 2>&1; echo "datasets rc=$?"; tail -3 $O/datasets.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --no-cpu-baseline --no-extra > $O/trace_bench.json 2> $O/trace.log
echo "trace rc=$?"
python3 tools/gs_fraction.py $O/trace $O/trace_bench.json > $O/gs_fraction.json; cat $O/gs_fraction.json
python3 tools/epoch_breakdown.py $O/trace > $O/breakdown.txt 2>&1; head -14 $O/breakdown.txt
