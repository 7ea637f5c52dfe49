#!/usr/bin/env bash
# Same-box A/B of fused-kernel builds: tools/ab_libs/libmmb_diag_<v>.so vs the current diag build
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
for v in head P cur; do
  lib=tools/ab_libs/libmmb_diag_$v.so; [ "$v" = cur ] && lib=tools/diag/libmmb_diag.so
  MMB_TOOLS_LIB=$PWD/$lib timeout -k 10 200 python tools/fused_shape_ab.py --rounds 2 --variants 0::2,0::1 > "$OUT/mosi_${v}_$rep.txt" 2>&1 || exit 1
  MMB_TOOLS_LIB=$PWD/$lib timeout -k 10 200 python tools/fused_shape_ab.py --T 40 --A 300 --Vd 300 --V 400000 --rounds 2 --variants 0::2 > "$OUT/main_${v}_$rep.txt" 2>&1 || exit 1
  echo "$v $rep: $(grep variant $OUT/mosi_${v}_$rep.txt | awk '{print $2, $4}' | tr '\n' ' ') main $(grep variant $OUT/main_${v}_$rep.txt | awk '{print $4}')"
done
done
