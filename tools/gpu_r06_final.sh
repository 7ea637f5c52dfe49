#!/usr/bin/env bash
# Round-6 final profile of the committed tree (TREE_SHA): part "trace" --
# rocprofv3 --kernel-trace --stats of the headline step (1M), the 125k
# per-rank step, the MOSI step and the POM workload; part "pmc" -- HBM
# traffic as separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md
# §HBM) of the synthetic, MOSI, ragged and POM workloads.  Each pass has its
# own time limit; the script stops at the first failure.
set -u
PART=${1:?trace or pmc}; TAG=${2:-r06final}
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
[ -f TREE_SHA ] && echo "tree: $(cat TREE_SHA)" > "$OUT/tree_sha.txt"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
cd /tmp
if [ "$PART" = trace ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.err"; ok $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace125k" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --utts 125000 --steps 20 --warmup 10 --only-main --no-cpu-baseline > "$OUT/trace125k_bench.json" 2> "$OUT/trace125k.err"; ok $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tracemosi" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --workload mosi --steps 10 --warmup 10 --only-main --no-cpu-baseline > "$OUT/tracemosi_bench.json" 2> "$OUT/tracemosi.err"; ok $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tracepom" -o run --output-format csv \
    -- python3 "$REPO/bench.py" --workload pom --steps 10 --warmup 5 --only-main --no-cpu-baseline > "$OUT/tracepom_bench.json" 2> "$OUT/tracepom.err"; ok $?
else
  for W in synthetic mosi ragged pom; do
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc_${W}_${C}" -o run --output-format csv \
        -- python3 "$REPO/bench.py" --workload $W --steps 2 --warmup 1 --only-main --no-cpu-baseline \
        > "$OUT/pmc_${W}_${C}.json" 2> "$OUT/pmc_${W}_${C}.err"; ok $?
    done
  done
fi
echo "final profile $PART $TAG done"
