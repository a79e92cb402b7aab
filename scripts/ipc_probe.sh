#!/bin/bash
# Peer-mapped exchange probe: N processes on this box's GPU(s), per allocation kind
# (0 hipMalloc, 1 fine-grained, 3 uncached); tools/ipc_probe.hip
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ipc_probe
mkdir -p $O
for kind in 3 1 0; do
  for world in 2 4; do
    d=$(mktemp -d)
    pids=()
    for r in $(seq 0 $((world - 1))); do
      timeout -k 5 60 tools/ipc_probe $r $world $d $kind > $O/k${kind}_w${world}_r$r.log 2>&1 &
      pids+=($!)
    done
    rc=0
    for p in "${pids[@]}"; do wait $p || rc=$?; done
    cat $O/k${kind}_w${world}_r*.log
    rm -rf $d
    [ $rc -eq 0 ] || { echo "probe kind $kind world $world rc=$rc"; exit $rc; }
  done
done
