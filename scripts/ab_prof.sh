#!/bin/bash
# Per-kernel A/B: rocprofv3 kernel stats of a short bench run for the in-tree build and each
# parallel-gcn_amd/<dir>/libpgcn.so.  usage: scripts/ab_prof.sh <dir>...   env: KPAT (kernel
# name pattern printed from the stats), BENCH_EXTRA
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
LIBS=("" "$@")
for d in "${LIBS[@]}"; do
  tag=${d:-default}
  lib=${d:+parallel-gcn_amd/$d/libpgcn.so}
  PGCN_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/abp_$tag" -o run -f csv -- \
      python3 bench.py --no-cpu-baseline --no-extra --steps 10 --warmup 3 ${BENCH_EXTRA:-} \
      > "gpurun_out/abp_$tag.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -5 "gpurun_out/abp_$tag.log"; exit $rc; }
  echo "== $tag $(grep -o '"value": [0-9.]*' "gpurun_out/abp_$tag.log" | head -1)"
  python3 - "gpurun_out/abp_$tag/run_kernel_stats.csv" "${KPAT:-xent}" <<'PY'
import csv, sys, re
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r['Name']):
        print(f"  {r['Name'][:70]:70s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.2f}")
PY
done
