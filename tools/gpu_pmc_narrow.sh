#!/usr/bin/env bash
# PMC passes (one rocprofv3 run each) over the two-kernel MOSI step with the
# narrow-frame stream kernel variants of the tools build:
#   bash tools/gpu_pmc_narrow.sh TAG "VARIANTS" ["CTRS" ...]
set -u
TAG=$1; VARS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1; echo "list rc=$?"
i=0
for V in $VARS; do
  for C in "$@"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/p${i}_v$V" -o run \
      --output-format csv -- python3 "$REPO/tools/narrow_ab.py" --variants $V --rounds 1 --steps 2 \
      > "$OUT/p${i}_v$V.txt" 2>&1
    rc=$?; echo "pass $i variant $V [$C] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
