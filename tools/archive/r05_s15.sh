# round 5 step 15: what bounds k_gsrb3 — kernel trace of C3 with the loads,
# the stores or both removed (timing-only builds; results are meaningless)
O=gpurun_out/r05/s15
mkdir -p $O
V=$PWD/octree-mg_amd/_variants
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in a3 a3ns a3nl a3nn; do
  OMG_LIB=$V/libomg_b3_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$v -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/$v.log 2>&1 || exit 1
  echo "== $v"; python tools/trace_by_grid.py $O/p_$v/run_kernel_trace.csv | grep -E "kernel|k_gsrb3"
done
