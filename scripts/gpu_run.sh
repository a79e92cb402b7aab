#!/bin/bash
# The one GPU-box runner (replaces the per-call scripts of rounds 4-5).  Every step runs under
# its own time limit and the runner stops at the first step that fails (a pytest run with
# failing tests -- rc 1 -- is reported and the next steps still run; a timeout, abort or fault
# ends the call).
#
# usage: scripts/gpu_run.sh <outdir under gpurun_out> <step> [<step> ...]
# steps (arguments after ':' are comma-separated and passed through):
#   pytest[:<pytest args>]     python -m pytest -m gpu -v <args, default tests> (no -x); '~' is
#                              a space inside an argument (-k,a~or~b)
#   smoke                      __graft_entry__.smoke()
#   bench:<tag>[:<args>]       bench.py <args> -> <tag>.json (+ .err)
#   g2:<tag>[:<args>]          bench.py --gpus 2 on this one GPU (PGCN_BENCH_SHARE_GPU=1)
#   rank[:<worlds>[,...]]      tools/rank_epoch.py (solo rank epochs, RANK_STEPS/RANK_WARMUP env)
#   datasets                   tools/datasets_bench.py (cora, citeseer, pubmed_synth)
#   trace:<tag>[:<args>]       rocprofv3 --kernel-trace --stats of bench.py --profile-only <args>,
#                              then tools/epoch_breakdown.py
#   dtrace:<tag>:<dataset>     rocprofv3 kernel trace of tools/datasets_bench.py on one dataset,
#                              then tools/epoch_breakdown.py (epochs between Adam launches)
#   rtrace:<tag>:<world>[:<knob=v,...>[:<library>]]  the same of tools/rank_epoch.py <world>
#                              (rank 0's solo epoch; knobs through RANK_KNOBS, an A/B build of
#                              the library through PGCN_LIB)
#   traffic:<tag>[:<args>[:<traffic.py args>]]  FETCH_SIZE / WRITE_SIZE passes (one counter
#                              group each) of the same, then tools/traffic.py (e.g.
#                              --epoch,11,--hidden,128+128+128,--write,r06)
#   tool:<tag>:<script>[:<args>] python3 tools/<script> <args> -> <tag>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
O=gpurun_out/${1:?outdir}
shift
mkdir -p "$O"
export TMPDIR=/tmp

args_of() { echo "${1//,/ }"; }
# the comma-separated list as an array in ARGV, '~' standing for a space inside one argument
# (pytest -k expressions)
argv_of() {
  ARGV=()
  local IFS=,
  local x
  for x in $1; do ARGV+=("${x//\~/ }"); done
}

run() {  # tag, seconds, command... (stdout -> tag.log)
  local tag=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$tag.log" 2>&1
  local rc=$?
  echo "[$tag] rc=$rc"
  tail -3 "$O/$tag.log" | cut -c1-300
  return $rc
}

for step in "$@"; do
  IFS=: read -r kind a b c d <<< "$step"
  case $kind in
    pytest)
      argv_of "${step#pytest:}"
      [ "$step" = pytest ] && ARGV=(tests)
      timeout -k 10 1500 python3 -u -m pytest -m gpu -v --timeout 300 \
          --timeout-method thread "${ARGV[@]}" > "$O/pytest.log" 2>&1
      rc=$?
      echo "[pytest] rc=$rc"
      grep -E "FAILED|ERROR" "$O/pytest.log" | head -20
      tail -2 "$O/pytest.log"
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)
      run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      timeout -k 10 900 python3 bench.py $(args_of "${b:-}") > "$O/$a.json" 2> "$O/$a.err"
      rc=$?
      echo "[bench $a] rc=$rc"
      cut -c1-400 "$O/$a.json"
      [ $rc -eq 0 ] || { tail -5 "$O/$a.err"; exit $rc; } ;;
    g2)
      PGCN_BENCH_SHARE_GPU=1 timeout -k 10 900 python3 bench.py --gpus 2 $(args_of "${b:-}") \
          > "$O/$a.json" 2> "$O/$a.err"
      rc=$?
      echo "[g2 $a] rc=$rc"
      cut -c1-400 "$O/$a.json"
      [ $rc -eq 0 ] || { tail -5 "$O/$a.err"; exit $rc; } ;;
    rank)
      timeout -k 10 900 python3 tools/rank_epoch.py "${a:-1,8}" > "$O/rank_epoch.json" \
          2> "$O/rank_epoch.err"
      rc=$?
      echo "[rank] rc=$rc"
      cat "$O/rank_epoch.err" | grep world
      [ $rc -eq 0 ] || exit $rc ;;
    datasets)
      run datasets 600 python3 tools/datasets_bench.py --out "$O/datasets.json" || exit $? ;;
    trace)
      ( cd /tmp && cd "$ROOT" && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
          -d "$O/$a" -o run -f csv -- python3 bench.py --profile-only $(args_of "${b:---steps,5,--warmup,2}") \
          > "$O/$a.log" 2>&1 )
      rc=$?
      echo "[trace $a] rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/$a.log"; exit $rc; }
      python3 tools/epoch_breakdown.py "$O/$a" > "$O/$a.breakdown.txt" 2>&1
      head -30 "$O/$a.breakdown.txt" ;;
    dtrace)  # dtrace:<tag>:<dataset>: kernel trace of tools/datasets_bench.py on one dataset
      ( cd /tmp && cd "$ROOT" && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
          -d "$O/$a" -o run -f csv -- python3 tools/datasets_bench.py --only "${b:-cora}" --graph 0 \
          --no-cpu --epochs 200 > "$O/$a.log" 2>&1 )
      rc=$?
      echo "[dtrace $a] rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/$a.log"; exit $rc; }
      python3 tools/epoch_breakdown.py "$O/$a" k_adam > "$O/$a.breakdown.txt" 2>&1
      head -30 "$O/$a.breakdown.txt" ;;
    rtrace)  # rtrace:<tag>:<world>[:<knob=v,...>[:<library>]]: kernel trace of tools/rank_epoch.py
      ( cd /tmp && cd "$ROOT" && RANK_KNOBS="${c:-}" PGCN_LIB="${d:+$ROOT/$d}" \
          timeout -k 10 600 rocprofv3 --kernel-trace --stats \
          -d "$O/$a" -o run -f csv -- python3 tools/rank_epoch.py "${b:-8}" > "$O/$a.log" 2>&1 )
      rc=$?
      echo "[rtrace $a] rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/$a.log"; exit $rc; }
      python3 tools/epoch_breakdown.py "$O/$a" k_adam > "$O/$a.breakdown.txt" 2>&1
      head -30 "$O/$a.breakdown.txt" ;;
    traffic)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        ( cd /tmp && cd "$ROOT" && timeout -s KILL 300 rocprofv3 --pmc $ctr -d "$O/$a/$ctr" -o run \
            -f csv -- python3 bench.py --profile-only $(args_of "${b:---steps,3,--warmup,1}") \
            > "$O/$a.$ctr.log" 2>&1 )
        rc=$?
        echo "[traffic $a $ctr] rc=$rc"
        [ $rc -eq 0 ] || { tail -20 "$O/$a.$ctr.log"; exit $rc; }
      done
      python3 tools/traffic.py "$O/$a" $(args_of "${c:-}") > "$O/$a.traffic.json" 2>&1
      cut -c1-600 "$O/$a.traffic.json" ;;
    tool)
      run "$a" 900 python3 "tools/$b" $(args_of "${c:-}") || exit $? ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
