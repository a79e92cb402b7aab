#!/bin/bash
# loss-kernel iteration: its GPU tests, the stamp timeline (ab_xst), the per-kernel A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "${PYTEST_K:-xent or exp_nonpos or output or reassociated or reddit_width or smoke}" > gpurun_out/ab_xent_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_xent_pytest.log; [ $rc -eq 0 ] || exit $rc
PGCN_LIB=parallel-gcn_amd/ab_xst/libpgcn.so timeout -k 10 300 python3 tools/xent_stamps.py > gpurun_out/xent_stamps.json 2> gpurun_out/xent_stamps.err
rc=$?; echo "stamps rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/xent_stamps.err; exit $rc; }
bash scripts/ab_prof.sh ${AB_LIBS:-ab_head}
