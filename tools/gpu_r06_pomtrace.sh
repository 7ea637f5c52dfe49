#!/usr/bin/env bash
set -u
OUT=$PWD/gpurun_out/r06pomtrace; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$REPO/tools/pom_graph_ab.py" --reps 5 --variants split_fork > "$OUT/ab.json" 2> "$OUT/ab.err"; echo "rc=$?"
cat "$OUT/ab.json"
