#!/usr/bin/env bash
set -u
OUT=$PWD/gpurun_out/r06probe; mkdir -p "$OUT"
for v in concurrent; do
  timeout -k 10 120 python3 tools/dbg/fork_graph_probe.py $v > "$OUT/$v.log" 2>&1; echo "$v rc=$?"; tail -1 "$OUT/$v.log"
done
timeout -k 10 300 python3 tools/split_ab.py > "$OUT/split_ab.json" 2> "$OUT/split_ab.err"; echo "ab rc=$?"
cat "$OUT/split_ab.json"
