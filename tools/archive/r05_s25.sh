# round 5 step 25: the new full-size periodic goldens (k_gsrb3 at its default
# bound: Helmholtz V-cycles, Laplacian FMG) through the Python path and the
# Fortran drop-in; the down-smoothing's last pass pushing colour 1 only
# (k_smooth_resid forms colour 0's ghosts): block3 tests, C3 timing
O=gpurun_out/r05/s25
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_fortran_dropin.py tests/test_gpu_block3.py -m gpu \
  -k "per256 or c3_per512 or block3 or per128 or per32" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  echo "== round $round" >> $O/ab.txt
  timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
done
grep -E "^==|^C3 " $O/ab.txt
