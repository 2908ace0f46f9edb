# round 5 step 46: k_gsrb3 loads rhs only where a substep's result is used (halo
# threads share a line): block3 tests, goldens, C3 A/B against every thread
# loading its own (tools/b3p_variants.py rhsall), kernel traces
O=gpurun_out/r05/s46
mkdir -p $O
R=$PWD
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_block3.py -m gpu > $O/pytest_block3.log 2>&1 || { tail -40 $O/pytest_block3.log; exit 1; }
grep -c PASSED $O/pytest_block3.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_fortran_dropin.py -m gpu \
  -k "per256 or c3_per512 or per128 or per32" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  for v in default rhsall; do
    echo "== round $round $v" >> $O/ab.txt
    if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
    timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
  done
done
unset OMG_LIB
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $R
for v in default rhsall; do
  if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/$v.log 2>&1 || exit 1
  echo "== $v" >> $O/by_grid.txt
  python tools/trace_by_grid.py $O/$v/run_kernel_trace.csv | grep -E "kernel|k_gsrb3" >> $O/by_grid.txt
done
unset OMG_LIB
cat $O/by_grid.txt
