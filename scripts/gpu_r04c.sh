#!/bin/bash
# r04 box 3: full GPU suite, A/B of the fused input-dropout kernel (wider workgroups), the
# edge-cut rank epochs with the one-chunk same-stream reduce-scatter, the W = 8 rank trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2 3; do
  for arm in nib0 nib1 old; do
    case $arm in
      nib0) env=""; k="--knob mask_nib=0" ;;
      nib1) env=""; k="--knob mask_nib=1" ;;
      old) env="PGCN_LIB=parallel-gcn_amd/ab_noxor3/libpgcn.so"; k="--knob mask_nib=0" ;;
    esac
    env $env timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra $k \
        > $O/ab_${arm}_$i.json 2> $O/ab_${arm}_$i.err || exit $?
    python3 -c "import json;d=json.load(open('$O/ab_${arm}_$i.json'));print('$arm', round(d['value'],1), round(d['value_unamortised'],1))"
  done
done
timeout -k 10 300 python3 tools/rank_epoch.py 1,2,4,8 0 16 > $O/rank_epoch.json 2> $O/rank_epoch.err || exit $?
cat $O/rank_epoch.json
RANK_KNOBS=xstream_ring=0 timeout -k 10 300 python3 tools/rank_epoch.py 8 0 16 > $O/rank_epoch_xs0.json 2> $O/rank_epoch_xs0.err || exit $?
echo "xstream_ring=0"; cat $O/rank_epoch_xs0.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rank8 -o run -f csv -- \
    python3 tools/rank_epoch.py 8 0 16 > $O/prof_rank8.log 2>&1; echo "rank8 trace rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/trace_bench.json 2> $O/trace.log
echo "trace rc=$?"
python3 tools/epoch_breakdown.py $O/trace > $O/breakdown.txt 2>&1; head -14 $O/breakdown.txt
python3 tools/gs_fraction.py $O/trace $O/trace_bench.json > $O/gs_fraction.json; cat $O/gs_fraction.json
timeout -k 10 400 python3 tools/datasets_bench.py --epochs 300 --graph 0 --out $O/datasets.json > $O/datasets.log 2>&1
echo "datasets rc=$?"; python3 -c "
import json; d=json.load(open('$O/datasets.json'))
for k,v in d.items():
    if isinstance(v, dict): print(k, round(v.get('eager_async_epochs_s',0),1), round(v.get('eager_frac_of_launch_floor',0),3))"
