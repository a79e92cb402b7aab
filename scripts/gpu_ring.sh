mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -v -x --timeout 120 --timeout-method thread -k "graphsum" > gpurun_out/t_ring.log 2>&1; rc=$?; tail -2 gpurun_out/t_ring.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/gs_ring_sweep.py 60,0,1,1 60,0,1,0 60,0,1,1 60,0,1,0 > gpurun_out/gs_ring_sweep.log 2>&1; rc=$?; tail -1 gpurun_out/gs_ring_sweep.log; exit $rc
