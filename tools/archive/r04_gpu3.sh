#!/bin/bash
# diagnose the GS smoothing with continuous BCs against the oracle; barrier probe
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 120 ./tools/xcd_probe > $O/xcd_probe.txt 2>&1; echo "xcd rc=$?" >> $O/xcd_probe.txt
timeout -k 10 600 python -u tools/diag_gsdbl.py "16 256 256 256 1 v gs lpl 0 c0 sol 1 lb 0" 2 > $O/diag_c0_2.txt 2>&1 || exit 1
