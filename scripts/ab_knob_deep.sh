#!/bin/bash
# 4-layer hidden-128 A/B of one engine knob on one box: bench lines with KNOB=0 and KNOB=1
# interleaved.  usage: KNOB=name scripts/ab_knob_deep.sh   env: ROUNDS, PYTEST_K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$PYTEST_K" > gpurun_out/abk_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/abk_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in 1 0; do
    timeout -k 10 400 python3 bench.py --hidden ${HIDDEN:-128,128,128} --steps 5 --warmup 1 --no-cpu-baseline --no-extra \
        --knob "$KNOB=$v" > "gpurun_out/abk_${v}_$r.json" 2> "gpurun_out/abk_${v}_$r.err"
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/abk_${v}_$r.json')); print('$KNOB=$v', round(d['value'],2), 'eps gs_ms', round(d['roofline']['avg_call_ms'],4), 'mfma', round(d['mfma']['frac'],3))" || { echo "bench rc=$rc"; tail -5 "gpurun_out/abk_${v}_$r.err"; exit 1; }
  done
done
