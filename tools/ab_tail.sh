export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo rc=$? >> gpurun_out/pytest_gpu.log
for round in 1 2; do
for v in tail0 tail1 default; do
  if [ $v = default ]; then unset OMG_LIB; else export OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_$v.so; fi
  echo "== $v round $round" >> gpurun_out/abtail.txt
  timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C1 C1-gsrb C2 C3 C4 C5-helm 2>&1 | tail -7 >> gpurun_out/abtail.txt || exit 1
done
done
unset OMG_LIB
OMG_TAIL_TIMING=1 timeout -k 10 200 python tools/configs_bench.py --no-cpu --only C1-gsrb > gpurun_out/tail_C1-gsrb.log 2>&1
OMG_TAIL_TIMING=1 timeout -k 10 200 python tools/configs_bench.py --no-cpu --only C3 > gpurun_out/tail_C3.log 2>&1
