# round 5 step 5: launch counts (C4, 4 loopback ranks, before/after the
# split-level fusions), the whole GPU suite, then one bench line
mkdir -p gpurun_out/r05
OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_r05_before.so timeout -k 10 120 python tools/c4_launch_counts.py 4 > gpurun_out/r05/s5_c4_launches_4ranks_before.txt 2>&1 || exit 1
timeout -k 10 120 python tools/c4_launch_counts.py 4 > gpurun_out/r05/s5_c4_launches_4ranks_after.txt 2>&1 || exit 1
paste gpurun_out/r05/s5_c4_launches_4ranks_before.txt gpurun_out/r05/s5_c4_launches_4ranks_after.txt | cut -c1-160
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05/s5_pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r05/s5_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r05/s5_bench.json 2> gpurun_out/r05/s5_bench.err
rc=$?
tail -c 600 gpurun_out/r05/s5_bench.json
exit $rc
