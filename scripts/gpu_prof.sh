#!/bin/bash
# Kernel trace + stats of the bench workload (rocprofv3), then the bench line itself.
# usage: scripts/gpu_prof.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-prof}; shift || true
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_trace" -o run -f csv -- \
    python3 bench.py --profile-only --steps 5 --warmup 1 "$@" > "gpurun_out/${TAG}_trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/${TAG}_trace.log"; exit $rc; }
python3 - "gpurun_out/${TAG}_trace" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.2f} %")
PY
