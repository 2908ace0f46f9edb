# round 5 step 11: three red-black substeps per pass (k_gsrb3) — periodic
# goldens bitwise, then C3 with and without OMG_NO_BLOCK3, and a kernel trace
O=gpurun_out/r05/s${STEP:-11}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_block3.py -m gpu \
  -k "per128 or c3_per512 or per32 or per64 or block3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  for sw in 1 0; do
    echo "== round $round OMG_NO_BLOCK3=$sw" >> $O/ab.txt
    OMG_NO_BLOCK3=$sw timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
  done
done
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-200
