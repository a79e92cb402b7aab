#!/bin/bash
# X-stream change: its GPU tests, then the per-kernel A/B (KPAT) against parallel-gcn_amd/<dirs>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "${PYTEST_K:-gemm_xstream or reddit_width or xstream or deep or fused}" > gpurun_out/ab_xs_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_xs_pytest.log; [ $rc -eq 0 ] || exit $rc
KPAT=${KPAT:-k_xs_} bash scripts/ab_prof.sh "$@"
