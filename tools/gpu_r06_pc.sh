#!/usr/bin/env bash
set -u
OUT=$PWD/gpurun_out/r06pc; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 120 python3 tools/pc_time.py > "$OUT/pc_time.json" 2> "$OUT/pc_time.err"; ok $?
cat "$OUT/pc_time.json"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_sif.py tests/test_gpu_robustness.py tests/test_gpu_split.py \
  "tests/test_gpu_variants.py::test_variants_agree[timeouts]" \
  tests/test_gpu_mmb2.py -k "pc or split or pom or mosi or full_size or graph or removal" > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
# last: may abort by design (HIP's missing-symbol path)
timeout -k 10 60 tools/dbg/missing_symbol_probe > "$OUT/missing_symbol.txt" 2>&1; echo "missing_symbol_probe rc=$?" >> "$OUT/missing_symbol.txt"
cat "$OUT/missing_symbol.txt"
