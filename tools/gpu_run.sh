#!/bin/bash
# Staged GPU session for gpurun: every GPU step has its own time limit; a
# crash, abort or time-out (exit >= 124, or 134/139) ends the session, plain
# test failures (exit 1) do not.
#   tools/gpu_run.sh "<stage> <stage> ..."   stages: smoke tests bench prof loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="${1:-smoke tests bench prof}"
rc_ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for s in $STAGES; do
  echo "=== stage $s $(date +%T)"
  case $s in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$? ;;
    tests) timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$? ;;
    prof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline) > gpurun_out/prof.log 2>&1; rc=$? ;;
    loop) { timeout -k 10 300 python tools/loopback_bench.py 8 128 5 0 && timeout -k 10 300 python tools/loopback_bench.py 8 128 5 && \
            timeout -k 10 300 python tools/loopback_bench.py 2 256 5 0 && timeout -k 10 300 python tools/loopback_bench.py 2 256 5; } > gpurun_out/loop.log 2>&1; rc=$? ;;
    *) echo "unknown stage $s"; rc=2 ;;
  esac
  echo "=== stage $s rc=$rc $(date +%T)"
  tail -5 gpurun_out/$s*.log 2>/dev/null
  if ! rc_ok $rc; then echo "stopping after $s (rc=$rc)"; exit $rc; fi
done
exit 0
