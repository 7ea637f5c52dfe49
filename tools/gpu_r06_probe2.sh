#!/usr/bin/env bash
# Round 6: the solve's phase marks (probe build) and the kernel trace of the
# 125k per-rank step (the solve's duration inside the step against alone).
set -u
OUT=$PWD/gpurun_out/${1:-r06probe2}; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 60 tools/pc_probe/pc_probe_mc > "$OUT/pc_probe.txt" 2>&1; ok $?
tail -6 "$OUT/pc_probe.txt"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace125k" -o run --output-format csv \
  -- python3 "$REPO/bench.py" --utts-per-gpu 125000 --only-main --no-cpu-baseline --steps 30 --warmup 10 > "$OUT/step125k.json" 2> "$OUT/step125k.err"); ok $?
f=$(ls "$OUT"/trace125k/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -12 "$f"
