#!/usr/bin/env bash
# Round-5 final profile of the committed tree (TREE_SHA): rocprofv3
# --kernel-trace --stats of the headline step (1M), the 125k per-rank step and
# the MOSI step; HBM traffic as separate FETCH_SIZE / WRITE_SIZE PMC passes
# (MI355X_MICROARCH.md §HBM) of the headline and MOSI steps; the MOSI step's
# L2 hits / misses (TCC_HIT_sum, TCC_MISS_sum) for its text-cache traffic.
# Each pass has its own time limit; the script stops at the first failure.
# (The 125k and MOSI passes warm up 10 steps: short steps after a model build
# otherwise time the chip's clock ramp, bench.py AUX_WARMUP_S.)
set -u
TAG=${1:-r05final}
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
[ -f TREE_SHA ] && echo "tree: $(cat TREE_SHA)" > "$OUT/tree_sha.txt"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; ok $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace125k" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --utts 125000 --steps 20 --warmup 10 --only-main --no-cpu-baseline > "$OUT/trace125k_bench.json" 2> "$OUT/trace125k.err"; ok $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tracemosi" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --workload mosi --steps 10 --warmup 10 --only-main --no-cpu-baseline > "$OUT/tracemosi_bench.json" 2> "$OUT/tracemosi.err"; ok $?
for W in synthetic mosi; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc_${W}_${C}" -o run --output-format csv \
      -- python3 "$REPO/bench.py" --workload $W --steps 2 --warmup 1 --only-main --no-cpu-baseline \
      > "$OUT/pmc_${W}_${C}.json" 2> "$OUT/pmc_${W}_${C}.err"; ok $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_mosi_TCC" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --workload mosi --steps 2 --warmup 1 --only-main --no-cpu-baseline \
  > "$OUT/pmc_mosi_TCC.json" 2> "$OUT/pmc_mosi_TCC.err"; ok $?
echo "final profile $TAG done"
