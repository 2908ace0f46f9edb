# round 5 step 21: k_gsrb3 as committed (4 planes ahead, levels of >= 4096
# boxes, columns shortened below 1024 workgroups) — parity, C3 A/B against
# one substep per launch, kernel trace, PMC of k_gsrb3 (bench's traffic)
O=gpurun_out/r05/s21
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_block3.py -m gpu \
  -k "per128 or c3_per512 or per32 or per64 or block3" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  for v in off main; do
    echo "== round $round $v" >> $O/ab.txt
    case $v in
      off) OMG_NO_BLOCK3=1 timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      main) timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
    esac
  done
done
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/prof.log 2>&1 || exit 1
python tools/trace_by_grid.py $O/prof/run_kernel_trace.csv > $O/by_grid.txt; head -10 $O/by_grid.txt
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "k_gsrb3" -d $GRAFT_REPO_ROOT/$O/p$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/configs_bench.py --no-cpu --only C3) > $O/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $O > $O/pmc_block3.json && echo pmc ok
