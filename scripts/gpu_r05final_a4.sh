#!/bin/bash
# r05 closing box A (fourth, at the last HEAD): full GPU suite, smoke(), the default bench line,
# leg + parity), the driver's window (20 after 5), the small datasets
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05final4
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20w5.json 2> $O/bench_s20w5.err; echo "bench20 rc=$?"; cut -c1-200 $O/bench_s20w5.json
timeout -k 10 400 python3 tools/datasets_bench.py --out $O/datasets.json > $O/datasets.log 2>&1; echo "datasets rc=$?"; tail -3 $O/datasets.log | cut -c1-200
