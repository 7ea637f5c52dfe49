#!/usr/bin/env bash
# PMC passes over tools/gram_one.py (one rocprofv3 run per counter set):
#   bash tools/gpu_pmc_gram.sh TAG "SHAPES" "CTRS" ["CTRS" ...]
set -u
TAG=$1; SHAPES=$2; shift 2
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
i=0
for S in $SHAPES; do
  for C in "$@"; do
    i=$((i + 1))
    MMB_GRAM_I8_SHAPE=$S timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/p${i}_s$S" -o run \
      --output-format csv -- python3 "$REPO/tools/gram_one.py" --reps 3 > "$OUT/p${i}_s$S.txt" 2>&1
    rc=$?; echo "pass $i shape $S [$C] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
