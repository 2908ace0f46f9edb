# round 5 step 22: the multi-rank tests first (drop-in under mpiexec, loopback),
# then the rest of the GPU suite
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fortran_dropin.py tests/test_gpu_multirank.py -m gpu -k "multirank" > gpurun_out/r05/s22_pytest_multirank.log 2>&1
rc=$?
tail -3 gpurun_out/r05/s22_pytest_multirank.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "not multirank" > gpurun_out/r05/s22_pytest_rest.log 2>&1
rc=$?
tail -3 gpurun_out/r05/s22_pytest_rest.log
exit $rc
