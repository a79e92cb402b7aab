#!/bin/bash
# r04 box 5: full GPU suite; A/B of the X-stream consumers' early epilogue / dZ loads against
# HEAD's build (ab_head); 8 rowsets per wave (lds_slots) on one GPU and on the edge-cut ranks'
# chunk graphs; stamped traffic passes of the ring sources.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
summ() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$2', round(d['value'],1), round(d['value_unamortised'],1), round(r['avg_call_ms']*1e3,1))"; }
for i in 1 2 3; do
  for arm in head new; do
    env=""; [ $arm = head ] && env="PGCN_LIB=parallel-gcn_amd/ab_head/libpgcn.so"
    env $env timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra \
        > $O/xs_${arm}_$i.json 2> $O/xs_${arm}_$i.err || exit $?
    summ $O/xs_${arm}_$i.json xs_$arm
  done
done
for i in 1 2; do
  for arm in s8b2 s8b4; do
    case $arm in
      s8b2) k="--knob lds_slots=8 --knob lds_blocks=2" ;;
      s8b4) k="--knob lds_slots=8 --knob lds_blocks=4" ;;
    esac
    timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra $k \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    summ $O/ab_${arm}_$i.json $arm
  done
done
export RANK_GS_PATHS="b4s16:lds_blocks=4,lds_slots=16,lds_min_kb=0;b4s8:lds_blocks=4,lds_slots=8,lds_min_kb=0;b2s8:lds_blocks=2,lds_slots=8,lds_min_kb=0;b8s8:lds_blocks=8,lds_slots=8,lds_min_kb=0"
timeout -k 10 300 python3 tools/rank_graphsum.py 2,4,8 1 > $O/rankgs_c1.json 2> $O/rankgs_c1.err; echo "c1 rc=$?"; tail -1 $O/rankgs_c1.json
timeout -k 10 300 python3 tools/rank_graphsum.py 2,4,8 2 > $O/rankgs_c2.json 2> $O/rankgs_c2.err; echo "c2 rc=$?"; tail -1 $O/rankgs_c2.json
unset RANK_GS_PATHS
timeout -k 10 300 python3 tools/rank_epoch.py 1,2,8 0 16 > $O/rank_epoch.json 2> $O/rank_epoch.err; echo "rank_epoch rc=$?"; cat $O/rank_epoch.json
RANK_KNOBS=rs_chunks=2,lds_slots=8 timeout -k 10 300 python3 tools/rank_epoch.py 2,8 0 16 > $O/rank_epoch_c2s8.json 2> $O/rank_epoch_c2s8.err
echo "rank_epoch c2 s8 rc=$?"; cat $O/rank_epoch_c2s8.json
bash scripts/gpu_traffic.sh r04e_traffic
