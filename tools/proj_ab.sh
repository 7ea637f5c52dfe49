#!/usr/bin/env bash
# A/B of the projection kernel variants (MMB_PROJ_VARIANT 0 = 32x32x16 tiles, 2 = pipelined 16x16x32,
# 1 = 16x16x32 tiles): the
# MMB2 GPU parity tests under variant $V (default 1), then the kernel
# microbench of each listed variant, twice, and the bench under each.
set -u
OUT=$PWD/gpurun_out/${TAG:-projab}; mkdir -p "$OUT"
MMB_PROJ_VARIANT=${V:-1} timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mmb2.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest (variant ${V:-1}) rc=$rc"; tail -3 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
for v in "$@" "$@"; do
  r=$(MMB_PROJ_VARIANT=$v timeout -k 10 300 python3 tools/kernel_bench.py project --reps 20 2>&1 | grep "project:") || exit 1
  echo "variant=$v $r"
done
for v in "$@"; do
  MMB_PROJ_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_v$v.json" 2> "$OUT/bench_v$v.err"
  rc=$?; [ "$rc" -eq 0 ] || { tail -3 "$OUT/bench_v$v.err"; exit "$rc"; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('variant', sys.argv[2], d['value'], d['ms_per_step'], d['phase_ms'])" "$OUT/bench_v$v.json" "$v"
done
