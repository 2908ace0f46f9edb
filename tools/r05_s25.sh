# round 5 step 25: the new full-size periodic goldens (k_gsrb3 at its default
# bound: Helmholtz V-cycles, Laplacian FMG) through the Python path and the
# Fortran drop-in
O=gpurun_out/r05/s25
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_fortran_dropin.py -m gpu \
  -k "per256 or c3_per512" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest.log | sed 's/.*:://'
