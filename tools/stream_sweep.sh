#!/usr/bin/env bash
# Sweep stream-kernel variants (MMB_STREAM_CFG) at the bench size.
for c in 0 1 2 3 4 5 6 7 8 9; do
  if [ "$c" = 0 ]; then unset MMB_STREAM_CFG; else export MMB_STREAM_CFG=$c; fi
  r=$(timeout -k 10 300 python3 tools/kernel_bench.py stream 2>&1 | grep "stream:") || exit 1
  echo "cfg=$c $r"
done
