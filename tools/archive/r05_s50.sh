# round 5 step 50: k_gsrb4 (four substeps per pass, the down-smoothing, then the
# unfused residual; OMG_BLOCK4): its tests, then C3 A/B and kernel traces
O=gpurun_out/r05/s50
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_block3.py -m gpu -k "block4" > $O/pytest_block4.log 2>&1 || { tail -40 $O/pytest_block4.log; exit 1; }
grep -c PASSED $O/pytest_block4.log
for round in 1 2; do
  for v in default OMG_BLOCK4; do
    echo "== round $round $v" >> $O/ab.txt
    if [ $v = default ]; then timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
    else env $v=1 timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1; fi
  done
done
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OMG_BLOCK4=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b4 -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/b4.log 2>&1 || exit 1
python tools/trace_by_grid.py $O/b4/run_kernel_trace.csv | head -14
