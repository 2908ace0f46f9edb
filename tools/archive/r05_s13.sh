# round 5 step 13: k_gsrb3 (pairs, two-box tiles, 32-bit offsets) — parity,
# then C3 A/B: one substep per launch / k_gsrb3 at 6 or 7 waves per SIMD
O=gpurun_out/r05/s${STEP:-13}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_block3.py -m gpu \
  -k "per128 or c3_per512 or per32 or per64 or block3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  for v in off main w7; do
    echo "== round $round $v" >> $O/ab.txt
    case $v in
      off) OMG_NO_BLOCK3=1 timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      main) timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      w7) OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_b3_w7.so timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
    esac
  done
done
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/prof.log 2>&1 || exit 1
python tools/trace_by_grid.py $O/prof/run_kernel_trace.csv | head -12
