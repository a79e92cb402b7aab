mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/gs_ring_diag.py > gpurun_out/gs_ring_diag.log 2>&1; rc=$?; tail -3 gpurun_out/gs_ring_diag.log; [ $rc -eq 0 ] || exit $rc
RING_WINDOW=1 timeout -k 10 300 python3 -u tools/gs_ring_diag.py > gpurun_out/gs_ring_diag1.log 2>&1; rc=$?; tail -3 gpurun_out/gs_ring_diag1.log; exit $rc
