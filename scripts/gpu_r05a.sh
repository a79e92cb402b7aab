#!/bin/bash
# r05 first box: the ADVICE fixes' tests, the full GPU suite, the default bench line, and the
# per-epoch ramp of the bench window (tools/epoch_ramp.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread \
  -k "test_gemm_xstream or hidden80 or above_128" > $O/pytest_advice.log 2>&1
rc=$?; echo "advice rc=$rc"; tail -3 $O/pytest_advice.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err; echo "bench rc=$?"; cut -c1-300 $O/bench_s20.json
timeout -k 10 300 python3 tools/epoch_ramp.py 40 > $O/ramp.json 2> $O/ramp.err; echo "ramp rc=$?"; python3 -c "import json;print(json.load(open('$O/ramp.json'))['summary'])"
