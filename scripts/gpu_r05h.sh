#!/bin/bash
# r05: one dropout state per group of chunks (mask_group) -- mask tests, epoch A/B (group by
# size / group 1 / by size + mask_side 1), the default epoch's kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05h
mkdir -p $O
ROOT=$(pwd)
timeout -k 10 400 python3 -u -m pytest -m gpu -v -x --timeout 150 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_engine.py -k "mask_side or mask_group or train_ahead or dropout or gemm_xstream" > $O/pytest_mask.log 2>&1
rc=$?; echo "mask tests rc=$rc"; grep -E "FAILED|ERROR" $O/pytest_mask.log | head -20; tail -2 $O/pytest_mask.log
[ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];m=d['mfma'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1), 'xs+gemm', round(m['ms_per_epoch']*1e3,1))"; }
for i in 1 2 3; do
  for arm in auto g1 side1; do
    k="--knob mask_group=0"; [ $arm = g1 ] && k="--knob mask_group=1"; [ $arm = side1 ] && k="--knob mask_side=1"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra $k \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- \
    python3 bench.py --profile-only --steps 20 --warmup 20 > $O/prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
S=$(find $O/prof -name run_kernel_stats.csv | head -1); head -14 $S | cut -c1-60,200-
