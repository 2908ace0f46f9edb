# round 5 step 35: builds of the library with one change each
# (tools/b3p_variants.py): subtract_rhs pass with nt stores (subnt), nt loads and stores (subntld); the plain k_gsrb3 pass at 6 waves per SIMD (occ6); C3 ms per cycle
O=gpurun_out/r05/s35
mkdir -p $O
R=$PWD
for round in 1 2; do
  for v in default subnt subntld occ6; do
    echo "== round $round $v" >> $O/ab.txt
    if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
    timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
  done
done
unset OMG_LIB
grep -E "^==|^C3 " $O/ab.txt
