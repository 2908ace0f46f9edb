# round 5 step 45: the RES pass loads old for the box columns only (halo threads
# share one line): block3 tests, goldens, C3 A/B against OMG_NO_BLOCK3R, trace
O=gpurun_out/r05/s45
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_block3.py -m gpu > $O/pytest_block3.log 2>&1 || { tail -40 $O/pytest_block3.log; exit 1; }
grep -c PASSED $O/pytest_block3.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_fortran_dropin.py -m gpu \
  -k "per256 or c3_per512 or per128 or per32" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  for v in default OMG_NO_BLOCK3R; do
    echo "== round $round $v" >> $O/ab.txt
    if [ $v = default ]; then timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
    else env $v=1 timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1; fi
  done
done
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/prof.log 2>&1 || exit 1
python tools/trace_by_grid.py $O/prof/run_kernel_trace.csv > $O/by_grid.txt; grep -E "kernel|k_gsrb3" $O/by_grid.txt
