#!/bin/bash
# r04 box 13: nibble-layout kernel walking tiles with a prefetch (GPU kernel tests, mask micro
# against HEAD's build); bench.py timed-region length on the same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for arm in head new; do
    env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
    env $env timeout -k 10 120 python3 tools/mask_micro.py > $O/micro_${arm}_$i.json 2> $O/micro_${arm}_$i.err || exit $?
    echo "$arm $(cat $O/micro_${arm}_$i.json)"
  done
done
bash scripts/gpu_warm.sh
