#!/usr/bin/env bash
set -u
OUT=$PWD/gpurun_out/r06split2; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_split.py > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python3 tools/split_ab.py --parts 1,2,3,4 > "$OUT/split_ab.json" 2> "$OUT/split_ab.err"; ok $?
cat "$OUT/split_ab.json"
