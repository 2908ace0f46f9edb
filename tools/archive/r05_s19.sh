# round 5 step 19: k_gsrb4r planes in flight: 2 (main) / 3 and 4 at 5 waves
# per SIMD (small spills) / 4 at its own register count; C3 and the trace
O=gpurun_out/r05/s19
mkdir -p $O
V=$PWD/octree-mg_amd/_variants
for round in 1 2; do
  for v in main b4a3w5 b4a4w5 b4a4; do
    echo "== round $round $v" >> $O/ab.txt
    case $v in
      main) timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      *) OMG_LIB=$V/libomg_b3_$v.so timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
    esac
  done
done
grep -E "^==|^C3 " $O/ab.txt
