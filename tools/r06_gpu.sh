#!/bin/bash
# round 6 GPU session: tag, then steps (smoke deep block3 c3multi loop bench suite), each
# under its own limit; stops at the first crash / abort / time-out
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
tag=$1; shift
O=gpurun_out/r06/${tag}
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for s in "$@"; do
  echo "=== $s $(date +%T)"
  case $s in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1; rc=$? ;;
    deep) timeout -k 10 900 $PT tests/test_gpu_multirank.py -k deep > ${O}_deep.log 2>&1; rc=$? ;;
    block3) timeout -k 10 900 $PT tests/test_gpu_block3.py > ${O}_block3.log 2>&1; rc=$? ;;
    golden) timeout -k 10 900 $PT tests/test_gpu_parity.py -k "test_device_matches_reference_golden and (c3_ or per256 or c2_256 or c5_)" > ${O}_golden.log 2>&1; rc=$? ;;
    c3multi) timeout -k 10 900 $PT tests/test_gpu_multirank.py -k c3_512 > ${O}_c3multi.log 2>&1; rc=$? ;;
    loop) { timeout -k 10 300 python tools/loopback_bench.py 2 512 5 && OMG_NO_DEEP=1 timeout -k 10 300 python tools/loopback_bench.py 2 512 5 && \
            timeout -k 10 300 python tools/loopback_bench.py 2 512 5 && OMG_NO_DEEP=1 timeout -k 10 300 python tools/loopback_bench.py 2 512 5; } > ${O}_loop.log 2>&1; rc=$? ;;
    mx) timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k mx > ${O}_mx.log 2>&1; rc=0 ;;
    physnx) timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_block3.py -k physical > ${O}_physnx.log 2>&1; rc=0 ;;
    phys) timeout -k 10 900 $PT tests/test_gpu_block3.py -k physical > ${O}_phys.log 2>&1; rc=$? ;;
    cfgab) { for v in "" OMG_NO_BLOCK3_PHYS=1 OMG_BLOCK4_PHYS=1 "" OMG_NO_BLOCK3_PHYS=1 OMG_BLOCK4_PHYS=1; do
               echo "== ${v:-default}"; env $v timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C2 C5-helm || exit 1; done; } > ${O}_cfgab.log 2>&1; rc=$? ;;
    smallab) { for v in "" OMG_BLOCK3_MIN_BOXES=512 OMG_BLOCK3_MIN_BOXES=64 "OMG_BLOCK3_MIN_BOXES=512 OMG_BLOCK3_SMALL_COL=4" \
                 "" OMG_BLOCK3_MIN_BOXES=512 OMG_BLOCK3_MIN_BOXES=64 "OMG_BLOCK3_MIN_BOXES=512 OMG_BLOCK3_SMALL_COL=4"; do
               echo "== ${v:-default}"; env $v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-parity || exit 1; done; } > ${O}_smallab.log 2>&1; rc=$? ;;
    c2prof) for v in default OMG_NO_BLOCK3_PHYS; do
              (cd /tmp && env $( [ $v = default ] || echo $v=1 ) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/${O}_c2prof_$v" -o run --output-format csv \
                 -- python3 "$GRAFT_REPO_ROOT/tools/configs_bench.py" --no-cpu --only C2) >> ${O}_c2prof.log 2>&1 || { rc=1; break; }; rc=0; done ;;
    phvar) { for r in 1 2; do for v in ${PHV:-default phnofix phnostore phnoload}; do
               echo "== $v"; if [ $v = default ]; then L=; else L=OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_$v.so; fi
               env $L timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C2 || exit 1; done; done; } > ${O}_phvar.log 2>&1; rc=$? ;;
    deferab) { for v in "" OMG_NO_DEFER_GC=1 "" OMG_NO_DEFER_GC=1; do
               echo "== ${v:-default}"; env $v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-parity || exit 1; done; } > ${O}_deferab.log 2>&1; rc=$? ;;
    sumsab) { for v in "" OMG_NO_FUSED_SUMS=1 "" OMG_NO_FUSED_SUMS=1 "" OMG_NO_FUSED_SUMS=1; do
               echo "== ${v:-default}"; env $v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-parity || exit 1; done; } > ${O}_sumsab.log 2>&1; rc=$? ;;
    sumsprof) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/${O}_sumsprof" -o run --output-format csv \
             -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-parity) > ${O}_sumsprof.log 2>&1; rc=$? ;;
    libab) { for r in 1 2; do for v in default ${LIBV:-head}; do
               echo "== $v"; if [ $v = default ]; then L=; else L=OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_$v.so; fi
               env $L timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-parity || exit 1; done; done; } > ${O}_libab.log 2>&1; rc=$? ;;
    c4prof) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/${O}_c4prof" -o run --output-format csv \
                 -- python3 "$GRAFT_REPO_ROOT/tools/configs_bench.py" --no-cpu --only C4) > ${O}_c4prof.log 2>&1; rc=$? ;;
    graphab) { for v in "" OMG_GRAPH=1 "" OMG_GRAPH=1; do
               echo "== ${v:-default}"; env $v timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C4 C2 C5-helm C1-gsrb || exit 1; done; } > ${O}_graphab.log 2>&1; rc=$? ;;
    smallab2) { for v in "" OMG_NO_SMALL3=1 "" OMG_NO_SMALL3=1; do
               echo "== ${v:-default}"; env $v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-parity || exit 1
               env $v timeout -k 10 300 python tools/configs_bench.py --no-cpu --only C2 C5-helm C1-gsrb || exit 1; done; } > ${O}_smallab2.log 2>&1; rc=$? ;;
    pmcb) timeout -k 10 900 bash tools/pmc.sh k_gsrb vcycle 3 > ${O}_pmcb.log 2>&1; rc=$? ;;
    configs) timeout -k 10 900 python tools/configs_bench.py --cpu-ranks 16 > ${O}_configs.log 2>&1; rc=$? ;;
    pmcc2) OUT=$PWD/gpurun_out/pmc_c2; mkdir -p $OUT; i=0; rc=0
           for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
                      "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
             i=$((i+1))
             (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_gsrb" -d "$OUT/p$i" -o pmc --output-format csv \
                -- python3 "$GRAFT_REPO_ROOT/tools/configs_bench.py" --no-cpu --only C2) > ${O}_pmcc2_p$i.log 2>&1 || { rc=1; break; }
           done ;;
    bench) timeout -k 10 600 python bench.py --no-cpu-baseline > ${O}_bench.json 2> ${O}_bench.err; rc=$? ;;
    suite) timeout -k 10 1100 $PT tests -m gpu > ${O}_pytest_gpu.log 2>&1; rc=$? ;;
    benchfull) timeout -k 10 600 python bench.py > ${O}_benchfull.json 2> ${O}_benchfull.err; rc=$? ;;
    prof) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/${O}_prof" -o run --output-format csv \
             -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-parity) > ${O}_prof.log 2>&1; rc=$? ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  echo "=== $s rc=$rc $(date +%T)"
  tail -3 ${O}_${s}*.log 2>/dev/null
  if [ $rc -ne 0 ]; then echo "stopping after $s (rc=$rc)"; exit $rc; fi
done
exit 0
