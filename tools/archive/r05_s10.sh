# round 5 step 10: the free-space GPU tests with the reverted one-wave tail
# (4aa12c0, OMG_TAIL_WAVE=1), as round 4's failing run had them
O=$PWD/gpurun_out/r05; mkdir -p $O
OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_r04_tailwave.so OMG_TAIL_WAVE=1 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_failures.py tests/test_gpu_free_space.py -m gpu > $O/s10_tailwave_free_space.log 2>&1
rc=$?
grep -E "PASSED|FAILED" $O/s10_tailwave_free_space.log | tail -30
exit 0
