#!/usr/bin/env bash
# Stream-kernel grid sweep: workgroups per CU (MMB_STREAM_GRID_MULT) of the
# grid-stride wave kernel, Zipf ids, kernel alone.
set -u
for m in 2 4 8 16 32 2 8; do
  r=$(MMB_STREAM_GRID_MULT=$m timeout -k 10 300 python3 tools/kernel_bench.py stream --reps 10 2>&1 | grep "stream:") || exit 1
  echo "grid_mult=$m $r"
done
