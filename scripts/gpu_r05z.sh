#!/bin/bash
# r05 late: the blocked d = 16 gather kernels on the dense reddit-114M graph (one call each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 300 python3 tools/gs_sparse.py 20 57307946 > $O/gs_dense.json 2> $O/gs_dense.err || exit $?
cat $O/gs_dense.json
