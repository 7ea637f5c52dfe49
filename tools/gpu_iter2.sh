#!/usr/bin/env bash
# Iteration run: SIF + MMB2 GPU tests, then bench --only-main for each listed
# workload (synthetic / ragged / pom), printing value, stream ms and phases.
set -u
OUT=$PWD/gpurun_out/${TAG:-iter2}; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sif.py tests/test_gpu_mmb2.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
for W in "$@"; do
  timeout -k 10 300 python3 bench.py --workload $W --steps 10 --warmup 3 --only-main --no-cpu-baseline > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  rc=$?; [ "$rc" -eq 0 ] || { tail -3 "$OUT/bench_$W.err"; exit "$rc"; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['phase_ms'])" "$OUT/bench_$W.json" "$W"
done
