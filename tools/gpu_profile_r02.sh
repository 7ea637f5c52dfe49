#!/usr/bin/env bash
# Round-2 profiling session (run via gpurun from the repo root):
#   1. every -m gpu test, smoke()
#   2. the default bench line (headline + configs_measured + CPU legs)
#   3. rocprofv3 --kernel-trace --stats of the headline bench (--only-main)
#   4. per workload (synthetic configs[3], ragged configs[3], POM configs[2]):
#      two separate PMC passes, FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md
#      §HBM: separate passes; gfx950 FETCH_SIZE counts half of wide reads)
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-r02}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
REPO=$PWD
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; ok $?
  tail -1 "$OUT/pytest.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok $?
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 600 python3 "$REPO/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"; ok $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['phase_ms'])" "$OUT/bench.json"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; ok $?
for W in synthetic ragged pom; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc_${W}_${C}" -o run --output-format csv \
      -- python3 "$REPO/bench.py" --workload $W --steps 2 --warmup 1 --only-main --no-cpu-baseline > "$OUT/pmc_${W}_${C}.json" 2> "$OUT/pmc_${W}_${C}.err"; ok $?
  done
done
echo "profiles done"
