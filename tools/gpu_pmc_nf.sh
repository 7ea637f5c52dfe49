#!/usr/bin/env bash
# PMC passes (one rocprofv3 run each) over tools/nf_ab.py with the narrow
# fused kernel builds of tools/ab_libs:
#   bash tools/gpu_pmc_nf.sh TAG "LIBTAGS" "CTRS" ["CTRS" ...]
set -u
TAG=$1; VARS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
i=0
for V in $VARS; do
  for C in "$@"; do
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -d "$OUT/p${i}_$V" -o run \
      --output-format csv -- python3 "$REPO/tools/nf_ab.py" --lib "$REPO/tools/ab_libs/libmmb_nf_$V.so" --steps 2 \
      > "$OUT/p${i}_$V.txt" 2>&1
    rc=$?; echo "pass $i $V [$C] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
