#!/bin/bash
# r04 box 7: input-dropout mask kernels -- the three-input-xor draw / advance build (ab_b1)
# against the in-tree build, alone (tools/mask_micro.py) and in the epoch, fused vs two launches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04g
mkdir -p $O
for arm in tree b1; do
  env=""; [ $arm != tree ] && env="PGCN_LIB=parallel-gcn_amd/ab_$arm/libpgcn.so"
  env $env timeout -k 10 120 python3 tools/mask_micro.py > $O/micro_$arm.json 2> $O/micro_$arm.err || exit $?
  echo "$arm $(cat $O/micro_$arm.json)"
done
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1))"; }
for i in 1 2 3; do
  for arm in tree_nib1 b1_nib1 b1_nib0; do
    case $arm in
      tree_nib1) env=""; k="" ;;
      b1_nib1) env="PGCN_LIB=parallel-gcn_amd/ab_b1/libpgcn.so"; k="" ;;
      b1_nib0) env="PGCN_LIB=parallel-gcn_amd/ab_b1/libpgcn.so"; k="--knob mask_nib=0" ;;
    esac
    env $env timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra $k \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
