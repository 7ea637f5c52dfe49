#!/usr/bin/env bash
# Round-4 trace session (same tree as the test + bench session):
# rocprofv3 --kernel-trace --stats of the headline step at 1M and at the
# 125k per-rank size, of the 1M MOSI step, then the MOSI PMC passes.
set -u
TAG=${1:-r04final}
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; ok $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace125k" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --utts 125000 --steps 20 --warmup 3 --only-main --no-cpu-baseline > "$OUT/trace125k_bench.json" 2> "$OUT/trace125k.err"; ok $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tracemosi" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --workload mosi --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/tracemosi_bench.json" 2> "$OUT/tracemosi.err"; ok $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc_mosi_${C}" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --workload mosi --steps 2 --warmup 1 --only-main --no-cpu-baseline \
    > "$OUT/pmc_mosi_${C}.json" 2> "$OUT/pmc_mosi_${C}.err"; ok $?
done
echo "trace session $TAG done"
