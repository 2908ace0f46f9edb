# round 5 step 26: k_gsrb3's correct_children form (correction + up-substeps
# 1-3 + coarse res in one pass): block3 tests, the periodic goldens, C3 A/B
O=gpurun_out/r05/s26
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_block3.py -m gpu > $O/pytest_block3.log 2>&1 || { tail -40 $O/pytest_block3.log; exit 1; }
grep -c PASSED $O/pytest_block3.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_fortran_dropin.py -m gpu \
  -k "per256 or c3_per512 or per128 or per32" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  echo "== round $round default" >> $O/ab.txt
  timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
  echo "== round $round OMG_NO_BLOCK3P=1" >> $O/ab.txt
  OMG_NO_BLOCK3P=1 timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
done
grep -E "^==|^C3 " $O/ab.txt
