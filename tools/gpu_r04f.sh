#!/usr/bin/env bash
# r04f: the narrow fused (MOSI-width) kernel, graph replays, then the MOSI leg.
set -o pipefail
OUT=gpurun_out/${1:-r04f}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_mmb2.py -x -v --timeout 300 --timeout-method thread \
  -k "narrow or compensated or mosi or real_pom or step_graph or full_size" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --workload mosi --only-main --no-cpu-baseline --steps 10 --warmup 3 \
  > "$OUT/mosi_main.json" 2> "$OUT/mosi_main.err" || exit $?
timeout -k 10 300 python3 -u bench.py --only-leg dataset_splits > "$OUT/splits.json" 2> "$OUT/splits.err" || exit $?
echo done
