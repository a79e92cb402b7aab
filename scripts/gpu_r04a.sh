#!/bin/bash
# r04 first box: the new parity tests, HEAD traffic/trace evidence, per-rank GraphSum shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_kernels.py tests/test_gpu_parity_large.py -m gpu -x -v \
    --timeout 300 --timeout-method thread -k "reddit_width or div_rn or exp_nonpos or loopback or edge_cut or dropout_mask or lds_graph or deep" > gpurun_out/r04a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/r04a_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_traffic.sh r04_head || exit $?
export RANK_GS_PATHS="b4:lds_blocks=4,lds_min_kb=0;b8:lds_blocks=8,lds_min_kb=0;b16:lds_blocks=16,lds_min_kb=0"
timeout -k 10 300 python3 tools/rank_graphsum.py 1,2,4,8 1 > gpurun_out/r04a_rankgs_c1.json 2> gpurun_out/r04a_rankgs_c1.err
echo "rankgs c1 rc=$?"; cat gpurun_out/r04a_rankgs_c1.json
timeout -k 10 300 python3 tools/rank_graphsum.py 2,4,8 2 > gpurun_out/r04a_rankgs_c2.json 2> gpurun_out/r04a_rankgs_c2.err
echo "rankgs c2 rc=$?"; cat gpurun_out/r04a_rankgs_c2.json
timeout -k 10 300 python3 tools/rank_epoch.py 1,2,8 0 16 > gpurun_out/r04a_rank_epoch.json 2> gpurun_out/r04a_rank_epoch.err
echo "rank_epoch rc=$?"; cat gpurun_out/r04a_rank_epoch.json; tail -4 gpurun_out/r04a_rank_epoch.err
