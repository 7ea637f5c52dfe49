#!/usr/bin/env bash
# HBM traffic passes (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 runs) over the bench step of each named workload:
#   bash tools/gpu_pmc_r04.sh TAG mosi synthetic ...
# then: python tools/summarize_pmc.py gpurun_out/TAG TAG mosi synthetic ...
set -u
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
for W in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc_${W}_${C}" -o run --output-format csv \
      -- python3 "$REPO/bench.py" --workload $W --steps 2 --warmup 1 --only-main --no-cpu-baseline \
      > "$OUT/pmc_${W}_${C}.json" 2> "$OUT/pmc_${W}_${C}.err"
    rc=$?; echo "pmc $W $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo "pmc done"
