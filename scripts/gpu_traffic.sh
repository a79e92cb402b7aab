#!/bin/bash
# HEAD evidence for the GraphSum roofline: a short bench line, the kernel trace (epoch
# breakdown = rocprof-sum fraction) and the FETCH_SIZE / WRITE_SIZE passes (traffic per call).
# usage: scripts/gpu_traffic.sh <outdir-name>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-r04_traffic}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra \
    > gpurun_out/$OUT.bench.json 2> gpurun_out/$OUT.bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/$OUT.bench.json; [ $rc -eq 0 ] || exit $rc
PASSES="trace fetch write" bash scripts/profile.sh $OUT || exit $?
python3 tools/traffic.py gpurun_out/$OUT > gpurun_out/$OUT.traffic.json || exit $?
cat gpurun_out/$OUT.traffic.json
python3 tools/epoch_breakdown.py gpurun_out/$OUT/trace > gpurun_out/$OUT.breakdown.txt 2>&1
head -3 gpurun_out/$OUT.breakdown.txt
