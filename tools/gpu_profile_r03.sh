#!/usr/bin/env bash
# Round-3 profiling session (run via gpurun from the repo root):
#   tools/gpu_profile_r03.sh TAG PART
#   PART a: every -m gpu test, smoke(), the default bench line, rocprofv3
#           --kernel-trace --stats of the headline bench (--only-main) at the
#           1M split and at the 125k per-rank size of the 8-GPU curve
#   PART b: per workload (synthetic configs[3], ragged configs[3], POM configs[2], MOSI configs[1]
#           configs[2]): separate PMC passes FETCH_SIZE and WRITE_SIZE
#           (MI355X_MICROARCH.md §HBM: separate passes; gfx950 FETCH_SIZE counts
#           half of wide reads), and rocprofv3 --kernel-trace --stats of the
#           e2e latent step (tools/latent_bench.py: word_zsum_kernel's time)
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:-r03}
PART=${2:-a}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
REPO=$PWD
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
if [ "$PART" = a ]; then
  if [ -z "${SKIP_TESTS:-}" ]; then
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; ok $?
    tail -1 "$OUT/pytest.log"
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok $?
    tail -1 "$OUT/smoke.log"
  fi
  timeout -k 10 600 python3 "$REPO/bench.py" --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; ok $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['phase_ms'])" "$OUT/bench.json"
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; ok $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace125k" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --utts 125000 --steps 20 --warmup 3 --only-main --no-cpu-baseline > "$OUT/trace125k_bench.json" 2> "$OUT/trace125k.err"; ok $?
else
  cd /tmp
  for W in synthetic ragged pom mosi; do
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 600 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc_${W}_${C}" -o run --output-format csv \
        -- python3 "$REPO/bench.py" --workload $W --steps 2 --warmup 1 --only-main --no-cpu-baseline > "$OUT/pmc_${W}_${C}.json" 2> "$OUT/pmc_${W}_${C}.err"; ok $?
    done
  done
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/latent" -o run --output-format csv \
    -- python3 "$REPO/tools/latent_bench.py" --steps 30 --cpu-steps 1 > "$OUT/latent_bench.json" 2> "$OUT/latent.err"; ok $?
fi
echo "profiles $PART done"
