# round 5 step 27: kernel trace of C3 with k_gsrb3's correct_children form
O=gpurun_out/r05/s27
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/configs_bench.py --no-cpu --only C3 > $O/prof.log 2>&1 || exit 1
python tools/trace_by_grid.py $O/prof/run_kernel_trace.csv > $O/by_grid.txt; head -24 $O/by_grid.txt
