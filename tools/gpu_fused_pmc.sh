#!/usr/bin/env bash
# PMC passes (one counter group per run) over the fused kernel's ablations.
set -u
TAG=${1:-fpmc}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
REPO=$PWD
cd /tmp
for V in "fused 0" "fused 1" "fused 2" "stream 0"; do
  set -- $V
  for C in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tagc=$(echo $C | tr ' ' '_')
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc_$1_$2_$tagc" -o run --output-format csv \
      -- python3 "$REPO/tools/fused_kernel_run.py" $1 --diag $2 --reps 2 > "$OUT/pmc_$1_$2_$tagc.log" 2>&1 || { echo "fail $V $C"; exit 1; }
  done
done
echo pmc done
