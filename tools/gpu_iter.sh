#!/usr/bin/env bash
# Iteration run: the MMB2 GPU tests, then the bench under each stream-kernel
# cache policy given (MMB_STREAM_POLICY values), no CPU leg.
set -u
OUT=$PWD/gpurun_out/${TAG:-iter}; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mmb2.py tests/test_gpu_sif.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
for p in "$@"; do
  MMB_STREAM_POLICY=$p timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_p$p.json" 2> "$OUT/bench_p$p.err"
  rc=$?; [ "$rc" -eq 0 ] || { tail -3 "$OUT/bench_p$p.err"; exit "$rc"; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('policy', sys.argv[2], d['value'], d['ms_per_step'], d['phase_ms'])" "$OUT/bench_p$p.json" "$p"
done
