#!/usr/bin/env bash
# GPU-box profiling session for one round (run via gpurun from the repo root).
#   1. the official bench line (default config: 1M utterances/GPU, 10 steps)
#   2. rocprofv3 --kernel-trace --stats of the same bench
#   3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of
#      the stream kernel (MI355X_MICROARCH.md §HBM: separate passes; gfx950
#      FETCH_SIZE counts half the bytes of wide coalesced reads)
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-r01}
STEPS=${STEPS:-10}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
REPO=$PWD
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }

timeout -k 10 900 python3 "$REPO/bench.py" --steps "$STEPS" --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"; ok $?
echo "bench: $(cat "$OUT/bench.json")"
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --steps "$STEPS" --warmup 3 --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; ok $?
timeout -k 10 900 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"; ok $?
timeout -k 10 900 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"; ok $?
echo "profiles done"
find "$OUT" -name "*.csv" | head -20
