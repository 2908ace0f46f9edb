#!/bin/bash
# per32_gsrb_v with the round-4 switches off one at a time
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "per32_gsrb_v or per64_gsrb_v or per128_box16 or c3_per512" > $O/diag_chain_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc: $(tail -1 $O/diag_chain_$tag.log)"
  [ $rc -le 1 ] || exit $rc
}
run default A=1
run nochain OMG_NO_RHS_CHAIN=1
run nofc OMG_NO_FILL_CRHS=1
run neither OMG_NO_RHS_CHAIN=1 OMG_NO_FILL_CRHS=1
exit 0
