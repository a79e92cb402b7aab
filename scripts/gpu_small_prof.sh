#!/bin/bash
# kernel traces of the small datasets' epochs (one dataset per rocprofv3 run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/small_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for d in cora citeseer pubmed_synth; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$d -o run -f csv -- \
      python3 tools/datasets_bench.py --epochs 200 --graph 0 --no-cpu --only $d > $O/$d.log 2>&1
  echo "$d rc=$?"
done
