# round 5 step 20: k_gsrb3 with its stage windows in LDS (73 VGPRs: three
# workgroups per CU at 4 planes ahead) — parity, then C3 A/B with 3 / 5 (at
# 6 waves per SIMD) / 6 planes ahead, and a trace
O=gpurun_out/r05/s20
mkdir -p $O
V=$PWD/octree-mg_amd/_variants
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_block3.py -m gpu \
  -k "per128 or c3_per512 or per32 or per64 or block3" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -c PASSED $O/pytest.log
for round in 1 2; do
  for v in main a3 a5w6 a6; do
    echo "== round $round $v" >> $O/ab.txt
    case $v in
      main) timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      *) OMG_LIB=$V/libomg_b3_$v.so timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
    esac
  done
done
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/prof.log 2>&1 || exit 1
python tools/trace_by_grid.py $O/prof/run_kernel_trace.csv > $O/by_grid.txt; head -8 $O/by_grid.txt
