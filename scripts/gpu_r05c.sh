#!/bin/bash
# r05: IPC probe, the peer-exchange tests (processes + loopback), the full GPU suite, the
# bench window with Â X last in the build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05c
mkdir -p $O
true
timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 150 --timeout-method thread \
  tests/test_gpu_peer_procs.py tests/test_gpu_multirank.py > $O/pytest_peer.log 2>&1
rc=$?; echo "peer tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/pytest_peer.log | head -30; tail -2 $O/pytest_peer.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_s20_$i.json 2> $O/bench_s20_$i.err; rc=$?; echo "bench rc=$rc"; cut -c1-200 $O/bench_s20_$i.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra > $O/bench_s100.json 2> $O/bench_s100.err; echo "bench100 rc=$?"; cut -c1-200 $O/bench_s100.json
timeout -k 10 300 python3 tools/epoch_ramp.py 40 > $O/ramp.json 2> $O/ramp.err; echo "ramp rc=$?"; python3 -c "import json;print(json.load(open('$O/ramp.json'))['summary'])"
