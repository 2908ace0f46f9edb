# round 5 step 48: the 20 x 12 against the 22 x 14 coarse tile again, the order
# reversed, three rounds, and two kernel traces of each
O=gpurun_out/r05/s48
mkdir -p $O
R=$PWD
for round in 1 2 3; do
  for v in ct22 default; do
    echo "== round $round $v" >> $O/ab.txt
    if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
    timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C3 >> $O/ab.txt 2>&1 || exit 1
  done
done
unset OMG_LIB
grep -E "^==|^C3 " $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $R
n=0
for v in ct22 default ct22 default; do
  if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$R/octree-mg_amd/_variants/libomg_b3p_$v.so; fi
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v$n -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/$v.log 2>&1 || exit 1
  echo "== $v" >> $O/by_grid.txt
  python tools/trace_by_grid.py $O/$v$n/run_kernel_trace.csv | grep -E "kernel|k_gsrb3" >> $O/by_grid.txt
done
unset OMG_LIB
cat $O/by_grid.txt
