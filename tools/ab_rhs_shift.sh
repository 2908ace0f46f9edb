cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2; do
  OMG_NO_RHS_SHIFT=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab_off_$i.log 2>&1 || exit $?
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab_on_$i.log 2>&1 || exit $?
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof_on" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-profile-pass) > gpurun_out/prof_on.log 2>&1
