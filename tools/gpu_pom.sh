#!/usr/bin/env bash
# POM-length stream-kernel iteration: the SIF + MMB2 GPU tests, then the
# configs[2] bench line (and the headline bench when FULL=1).
set -u
OUT=$PWD/gpurun_out/${TAG:-pom}; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sif.py tests/test_gpu_mmb2.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 300 python3 bench.py --workload pom --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/pom.json" 2> "$OUT/pom.err"
rc=$?; echo "pom rc=$rc"; [ "$rc" -eq 0 ] || { tail -3 "$OUT/pom.err"; exit "$rc"; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['phase_ms'])" "$OUT/pom.json"
[ -n "${FULL:-}" ] || exit 0
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ "$rc" -eq 0 ] || { tail -3 "$OUT/bench.err"; exit "$rc"; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['phase_ms'], d.get('stream_uniform_ids'))" "$OUT/bench.json"
