#!/bin/bash
# A/B bench on one box: GPU tests matching $PYTEST_K (if set), then the default bench and one
# bench per knob set in $AB ("k=v,k=v;k=v" ...), all without the CPU leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_ab.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
IFS=';' read -ra SETS <<< "${AB:-}"
for set in "" "${SETS[@]}"; do
  args=""
  IFS=',' read -ra KV <<< "$set"
  for kv in "${KV[@]}"; do [ -n "$kv" ] && args="$args --knob $kv"; done
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline $args ${BENCH_EXTRA:-} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$i.json')); print('[$set]', round(d['value'],1), 'eps', 'gs_ms', round(d['roofline']['avg_call_ms'],4), 'frac', round(d['roofline']['frac'],3))" || { echo "bench rc=$rc"; tail -5 gpurun_out/ab_$i.err; exit 1; }
  i=$((i+1))
done
