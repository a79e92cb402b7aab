#!/bin/bash
# GraphSum A/B on one box: the GraphSum GPU tests against the in-tree build, then per build
# (in-tree, then parallel-gcn_amd/<dir>/ for each dir) tools/gs_call.py at d = 16 and d = 128,
# then interleaved bench lines.  usage: scripts/ab_ring.sh <dir>...   env: ROUNDS, PYTEST_K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "${PYTEST_K:-graphsum or lds_graph or reddit_width}" > gpurun_out/ab_ring_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_ring_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS=("" "$@")
for d in "${LIBS[@]}"; do
  tag=${d:-default}
  lib=${d:+parallel-gcn_amd/$d/libpgcn.so}
  for w in 16 128; do
    PGCN_LIB=$lib timeout -k 10 200 python3 tools/gs_call.py 20 $w > "gpurun_out/ab_gs_${tag}_$w.json" 2> "gpurun_out/ab_gs_${tag}_$w.err"
    rc=$?; [ $rc -eq 0 ] || { echo "$tag gs_call rc=$rc"; tail -5 "gpurun_out/ab_gs_${tag}_$w.err"; exit $rc; }
    echo "$tag d=$w $(cat gpurun_out/ab_gs_${tag}_$w.json)"
  done
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for d in "${LIBS[@]}"; do
    tag=${d:-default}
    lib=${d:+parallel-gcn_amd/$d/libpgcn.so}
    PGCN_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra ${BENCH_EXTRA:-} \
        > "gpurun_out/ab_${tag}_$r.json" 2> "gpurun_out/ab_${tag}_$r.err"
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${tag}_$r.json')); print('$tag', round(d['value'],1), 'eps gs_ms', round(d['roofline']['avg_call_ms'],4), 'frac', round(d['roofline']['frac'],3))" || { echo "$tag bench rc=$rc"; tail -5 "gpurun_out/ab_${tag}_$r.err"; exit 1; }
  done
done
