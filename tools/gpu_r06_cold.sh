#!/usr/bin/env bash
# Round 6: the solve's phase marks warm (back to back) and cold (a 1 GiB copy
# kernel before each solve).
set -u
OUT=$PWD/gpurun_out/${1:-r06cold}; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 60 tools/pc_probe/pc_probe_mc > "$OUT/pc_probe_warm.txt" 2>&1; ok $?
timeout -k 10 60 tools/pc_probe/pc_probe_mc cold > "$OUT/pc_probe_cold.txt" 2>&1; ok $?
grep "rep 4" "$OUT/pc_probe_warm.txt"; grep "rep 4" "$OUT/pc_probe_cold.txt"
