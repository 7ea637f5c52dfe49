#!/usr/bin/env bash
for d in zipf uniform hot seq; do
  r=$(timeout -k 10 300 python3 tools/kernel_bench.py stream --ids $d 2>&1 | grep "stream:") || exit 1
  echo "ids=$d $r"
done
