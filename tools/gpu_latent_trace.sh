#!/usr/bin/env bash
# rocprofv3 kernel trace of the graph latent step alone
set -u
TAG=${1:-latent_trace}
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$REPO/tools/latent_bench.py" --only-graph --steps 200 > "$OUT/bench.json" 2> "$OUT/err.txt"
rc=$?; cat "$OUT/bench.json"; exit $rc
