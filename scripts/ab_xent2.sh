#!/bin/bash
# loss-kernel change: its GPU tests, then the per-kernel A/B against parallel-gcn_amd/ab_head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "${PYTEST_K:-xent or output or reassociated or reddit_width or smoke}" > gpurun_out/ab_xent_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_xent_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_prof.sh ${AB_LIBS:-ab_head}
