# round 5 step 9: the reverted one-wave tail (4aa12c0) on free128_box16_f,
# OMG_TAIL_WAVE=1 against the workgroup tail, at 4 and 1 loopback ranks
O=$PWD/gpurun_out/r05/s9
mkdir -p $O
export OMG_LIB=$PWD/octree-mg_amd/_variants/libomg_r04_tailwave.so
for r in 4 1; do
  OMG_TAIL_WAVE=1 timeout -k 10 180 python tools/tailwave_diag.py $O/w$r.npz $r > $O/w$r.log 2>&1 || exit 1
  timeout -k 10 180 python tools/tailwave_diag.py $O/g$r.npz $r > $O/g$r.log 2>&1 || exit 1
  echo "== $r ranks: one-wave (first) against workgroup tail" >> $O/cmp.txt
  python tools/tailwave_cmp.py $O/w$r.npz $O/g$r.npz >> $O/cmp.txt
done
cat $O/cmp.txt
rm -f $O/*.npz
