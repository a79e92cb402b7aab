#!/bin/bash
# A/B of library builds on one box: per build (in-tree default, then parallel-gcn_amd/<dir>/
# for each dir argument) a kernel trace of the bench workload (per-kernel averages of the
# kernels matching $KERNELS), then the bench lines interleaved A B .. A B ($ROUNDS rounds).
# usage: scripts/ab_libs.sh <dir>...      env: KERNELS (regex), ROUNDS, BENCH_EXTRA
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROOT=$(pwd)
LIBS=("" "$@")
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for d in "${LIBS[@]}"; do
  tag=${d:-default}
  lib=${d:+parallel-gcn_amd/$d/libpgcn.so}
  PGCN_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/ab_$tag" -o run -f csv -- \
      python3 bench.py --profile-only --steps 4 --warmup 1 ${BENCH_EXTRA:-} > "gpurun_out/ab_${tag}_trace.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$tag trace rc=$rc"; tail -5 "gpurun_out/ab_${tag}_trace.log"; exit $rc; }
  python3 - "gpurun_out/ab_$tag" "$tag" "${KERNELS:-.}" <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    n = r["Kernel_Name"].split("(")[0][-60:]
    if re.search(sys.argv[3], n):
        by.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in by.items():
    print(f"{sys.argv[2]:10s} {n:60s} n={len(v):3d} avg={sum(v)/len(v):8.2f} us  last6={[round(x,1) for x in v[-6:]]}")
PY
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for d in "${LIBS[@]}"; do
    tag=${d:-default}
    lib=${d:+parallel-gcn_amd/$d/libpgcn.so}
    PGCN_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra ${BENCH_EXTRA:-} \
        > "gpurun_out/ab_${tag}_$r.json" 2> "gpurun_out/ab_${tag}_$r.err"
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${tag}_$r.json')); print('$tag', round(d['value'],1), 'eps gs_ms', round(d['roofline']['avg_call_ms'],4))" || { echo "$tag bench rc=$rc"; tail -5 "gpurun_out/ab_${tag}_$r.err"; exit 1; }
  done
done
