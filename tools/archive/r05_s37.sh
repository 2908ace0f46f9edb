# round 5 step 37: kernel traces of the store-wave bound builds (nostw, nopush:
# their results differ, so only the k_gsrb3 kernels' own times are read)
O=gpurun_out/r05/s37
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
for v in default nostw nopush; do
  if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/$v.log 2>&1 || exit 1
  echo "== $v" >> $O/by_grid.txt
  python tools/trace_by_grid.py $O/$v/run_kernel_trace.csv | grep -E "kernel|k_gsrb3" >> $O/by_grid.txt
done
unset OMG_LIB
cat $O/by_grid.txt
