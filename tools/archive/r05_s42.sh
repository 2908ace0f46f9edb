# round 5 step 42: k_gsrb3 with 2 / 6 planes of loads in flight (tools/b3p_variants.py
# a2, a6; a2 has 65-82 VGPRs, three workgroups per CU): C3 interleaved, traces
O=gpurun_out/r05/s42
mkdir -p $O
R=$PWD
for round in 1 2; do
  for v in default a2 a6; do
    echo "== round $round $v" >> $O/ab.txt
    if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
    timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
  done
done
unset OMG_LIB
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $R
for v in default a2 a6; do
  if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/$v.log 2>&1 || exit 1
  echo "== $v" >> $O/by_grid.txt
  python tools/trace_by_grid.py $O/$v/run_kernel_trace.csv | grep -E "kernel|k_gsrb3" >> $O/by_grid.txt
done
unset OMG_LIB
cat $O/by_grid.txt
