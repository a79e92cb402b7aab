#!/bin/bash
# r04 box 12: kernel traces of the small datasets' epochs, HEAD's build (ab_head) vs the
# in-tree build (sparse-X SpMM / plain GraphSum tail / reduce loads), then longer epoch runs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for arm in head new; do
  for d in cora pubmed_synth; do
    if [ $arm = head ]; then
      PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${arm}_$d -o run -f csv -- \
          python3 tools/datasets_bench.py --epochs 300 --graph 0 --no-cpu --only $d > $O/${arm}_$d.log 2>&1
    else
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${arm}_$d -o run -f csv -- \
          python3 tools/datasets_bench.py --epochs 300 --graph 0 --no-cpu --only $d > $O/${arm}_$d.log 2>&1
    fi
    echo "$arm $d rc=$?"
  done
done
for i in 1 2 3; do
  for arm in head new; do
    env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
    env $env timeout -k 10 300 python3 tools/datasets_bench.py --epochs 2000 --graph 0 --no-cpu --out $O/ds_${arm}_$i.json > $O/ds_${arm}_$i.log 2>&1 || exit $?
    python3 -c "
import json; d=json.load(open('$O/ds_${arm}_$i.json'))
print('$arm', ' '.join(f'{k} {v.get(\"eager_async_epochs_s\",0):.0f}' for k,v in d.items() if isinstance(v, dict)))"
  done
done
