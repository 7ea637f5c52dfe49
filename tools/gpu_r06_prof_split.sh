#!/usr/bin/env bash
set -u
OUT=$PWD/gpurun_out/r06profsplit; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
for P in 2 4; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/p$P" -o run --output-format csv \
  -- python3 "$REPO/tools/split_ab.py" --parts $P --reps 10 > "$OUT/p$P.json" 2> "$OUT/p$P.err"; echo "p$P rc=$?"
done
