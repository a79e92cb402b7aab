#!/bin/bash
# bench.py timed region length: 20 steps after 3 warmup epochs vs 100 after 20 (same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/warm
mkdir -p $O
for i in 1 2; do
  for arm in s20w3 s100w20 s200w50; do
    case $arm in s20w3) a="--steps 20 --warmup 3";; s100w20) a="--steps 100 --warmup 20";; s200w50) a="--steps 200 --warmup 50";; esac
    timeout -k 10 300 python3 bench.py $a --no-cpu-baseline --no-extra > $O/${arm}_$i.json 2> $O/${arm}_$i.err || exit $?
    python3 -c "import json;d=json.load(open('$O/${arm}_$i.json'));print('$arm', round(d['value'],1), round(d['value_unamortised'],1), round(d['ms_per_step'],4))"
  done
done
