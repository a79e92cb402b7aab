#!/bin/bash
# r05: bench.py --gpus 8 rehearsal (8 rank processes sharing one GPU, peer exchange over hipIpc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05w
mkdir -p $O
PGCN_BENCH_SHARE_GPU=1 timeout -k 10 900 python3 bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $O/bench_g8.json 2> $O/bench_g8.err; rc=$?; echo "gpus 8 rc=$rc"; cut -c1-300 $O/bench_g8.json; tail -5 $O/bench_g8.err; exit $rc
