mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/gs_ring_sweep.py 60,1,1 60,0,1 0,1,1 0,0,1 40,1,1 100,1,1 60,2,1 > gpurun_out/gs_ring_sweep.log 2>&1; rc=$?; tail -1 gpurun_out/gs_ring_sweep.log; exit $rc
