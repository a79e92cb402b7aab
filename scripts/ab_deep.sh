#!/bin/bash
# 4-layer hidden-128 A/B on one box: bench lines (BASELINE configs[4] at one GPU) of the in-tree
# build and parallel-gcn_amd/<dir>/ builds, interleaved.  usage: scripts/ab_deep.sh <dir>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=("" "$@")
for r in $(seq 1 ${ROUNDS:-2}); do
  for d in "${LIBS[@]}"; do
    tag=${d:-default}
    lib=${d:+parallel-gcn_amd/$d/libpgcn.so}
    PGCN_LIB=$lib timeout -k 10 400 python3 bench.py --hidden 128,128,128 --steps 5 --warmup 1 \
        --no-cpu-baseline --no-extra > "gpurun_out/abd_${tag}_$r.json" 2> "gpurun_out/abd_${tag}_$r.err"
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/abd_${tag}_$r.json')); print('$tag', round(d['value'],2), 'eps', 'mfma', round(d['mfma']['frac'],3), round(d['mfma']['ms_per_epoch'],3), 'ms', 'gs_ms', round(d['roofline']['avg_call_ms'],4))" || { echo "$tag bench rc=$rc"; tail -5 "gpurun_out/abd_${tag}_$r.err"; exit 1; }
  done
done
