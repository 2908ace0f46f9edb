# round 5: the GPU suite (and, when given, extra steps), each under its own limit
mkdir -p gpurun_out/r05
tag=${1:-s2}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05/${tag}_pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r05/${tag}_pytest_gpu.log
exit $rc
