#!/usr/bin/env bash
# Stream-kernel cache-policy sweep (MMB_STREAM_POLICY bits: 1 NT frame loads,
# 2 NT output stores, 4 four-frame load groups), zipf and uniform token ids.
set -u
for ids in zipf uniform; do
  for p in 0 1 2 3 4 5 6 7; do
    r=$(MMB_STREAM_POLICY=$p timeout -k 10 300 python3 tools/kernel_bench.py stream --ids $ids --reps 10 2>&1 | grep "stream:") || exit 1
    echo "ids=$ids policy=$p $r"
  done
done
