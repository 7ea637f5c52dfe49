#!/usr/bin/env bash
# int8-Gram session: MMB2 + SIF GPU tests, then kernel timings and a bench A/B (MMB_GRAM=f64 vs default).
set -u
OUT=$PWD/gpurun_out/${TAG:-gi8}; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mmb2.py tests/test_gpu_sif.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 300 python3 tools/kernel_bench.py stream stream_cm gram gram_i8 --reps 10 > "$OUT/kb.log" 2>&1; rc=$?; grep -v amdgpu.ids "$OUT/kb.log"; [ "$rc" -eq 0 ] || exit "$rc"
for g in f64 i8 f64 i8; do
  MMB_GRAM=$g timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/bench_$g.json" 2> "$OUT/bench_$g.err"
  rc=$?; [ "$rc" -eq 0 ] || { tail -3 "$OUT/bench_$g.err"; exit "$rc"; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('gram', sys.argv[2], d['value'], d['ms_per_step'], d['phase_ms'])" "$OUT/bench_$g.json" "$g"
done
