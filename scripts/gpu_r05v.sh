#!/bin/bash
# r05: bench.py --gpus 2 / 4 end to end on one GPU (PGCN_BENCH_SHARE_GPU=1 rehearsal)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 600 --timeout-method thread \
  tests/test_gpu_bench_procs.py > $O/pytest.log 2>&1
rc=$?; echo "bench procs test rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
PGCN_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 bench.py --gpus 4 --steps 10 --warmup 3 --no-cpu-baseline --no-extra > $O/bench_g4.json 2> $O/bench_g4.err; echo "gpus 4 rc=$?"; cut -c1-400 $O/bench_g4.json
