set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gs_micro.py > gpurun_out/gs_micro.json 2> gpurun_out/gs_micro.err && \
timeout -k 10 200 python3 tools/gs_stamps.py > gpurun_out/gs_stamps.json 2> gpurun_out/gs_stamps.err && \
PASSES="fetch write" bash scripts/profile.sh r01_pmc_lds
rc=$?; cat gpurun_out/gs_micro.json gpurun_out/gs_stamps.json; exit $rc
