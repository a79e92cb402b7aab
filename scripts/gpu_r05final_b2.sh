#!/bin/bash
# r05 closing box B2 (at the last HEAD): the reddit-11.6M and 4-layer bench lines, the --gpus 2
# rehearsal on one GPU (two rank processes over the peer exchange)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05final_b2
mkdir -p $O
timeout -k 10 600 python3 bench.py --workload reddit-11.6M > $O/bench_11.6M.json 2> $O/bench_11.6M.err; rc=$?; echo "11.6M rc=$rc"; cut -c1-200 $O/bench_11.6M.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py --hidden 128,128,128 --steps 20 --warmup 5 > $O/bench_4layer.json 2> $O/bench_4layer.err; rc=$?; echo "4layer rc=$rc"; cut -c1-200 $O/bench_4layer.json; [ $rc -eq 0 ] || exit $rc
PGCN_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-extra > $O/bench_g2.json 2> $O/bench_g2.err; rc=$?; echo "g2 rc=$rc"; cut -c1-300 $O/bench_g2.json
