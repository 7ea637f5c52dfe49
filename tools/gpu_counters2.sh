#!/usr/bin/env bash
# rocprofv3 -L listing, then counter passes on one kernel_bench kernel.
#   bash tools/gpu_counters2.sh TAG KERNEL "CTR ..." ["CTR ..." ...]
set -u
TAG=$1; K=$2; shift 2
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1; echo "list rc=$?"
cd "$REPO"
bash tools/gpu_counters.sh "$TAG" "$K" "$@"
