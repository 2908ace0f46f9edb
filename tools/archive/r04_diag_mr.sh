#!/bin/bash
# localise the 4-rank c1_gsrb_f_maxres mismatch: default, no mid kernel, no
# fused physical-face down-step (a test failure continues, anything else stops)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_multirank.py \
    -k "c1_gsrb_f_maxres or per32_gsrb_v or c4_ref2_box16_gsrb" > $O/diag_mr_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc: $(tail -1 $O/diag_mr_$tag.log)"
  [ $rc -le 1 ] || exit $rc
}
run default A=1
run nomid OMG_NO_MID=1
run nobc OMG_NO_FUSE_DOWN_BC=1
run neither OMG_NO_MID=1 OMG_NO_FUSE_DOWN_BC=1
exit 0
