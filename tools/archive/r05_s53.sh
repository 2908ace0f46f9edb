# round 5 step 53: the clean rebuild of the final tree — block3 / block4 tests,
# the periodic goldens, smoke
O=gpurun_out/r05/s53
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_block3.py tests/test_gpu_parity.py -m gpu -k "block or per256 or c3_per512" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
