# round 5 step 4: C4 launch counts at 4 loopback ranks before/after the
# split-level fusions, then the multi-rank GPU tests (loopback + MPI drop-in)
mkdir -p gpurun_out/r05
OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_r05_before.so timeout -k 10 120 python tools/c4_launch_counts.py 4 > gpurun_out/r05/s4_c4_launches_4ranks_before.txt 2>&1 || exit 1
timeout -k 10 120 python tools/c4_launch_counts.py 4 > gpurun_out/r05/s4_c4_launches_4ranks_after.txt 2>&1 || exit 1
paste gpurun_out/r05/s4_c4_launches_4ranks_before.txt gpurun_out/r05/s4_c4_launches_4ranks_after.txt | cut -c1-160
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_fortran_dropin.py -m gpu > gpurun_out/r05/s4_pytest_multirank.log 2>&1
rc=$?
tail -3 gpurun_out/r05/s4_pytest_multirank.log
exit $rc
