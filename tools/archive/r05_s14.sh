# round 5 step 14: k_gsrb3 loads in flight — C3 with 2 / 3 / 4 planes ahead
# (and 3 ahead at 6 waves per SIMD) against one substep per launch
O=gpurun_out/r05/s14
mkdir -p $O
V=$PWD/octree-mg_amd/_variants
for round in 1 2; do
  for v in off a2 a3 a3w6 a4; do
    echo "== round $round $v" >> $O/ab.txt
    case $v in
      off) OMG_NO_BLOCK3=1 timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      a2) timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
      *) OMG_LIB=$V/libomg_b3_$v.so timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1 ;;
    esac
  done
done
grep -E "^==|^C3 " $O/ab.txt
