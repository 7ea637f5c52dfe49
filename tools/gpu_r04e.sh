#!/usr/bin/env bash
# r04e: the regressor (multi-workgroup training kernel, in-launch validation)
# and the per-split legs.  Each GPU step under its own time limit.
set -o pipefail
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_regressor.py tests/test_gpu_mmb2.py -x -v \
  --timeout 300 --timeout-method thread -k "regressor or real_pom or mosi_splits or step_graph" \
  > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --only-leg regressor > "$OUT/regressor.json" 2> "$OUT/regressor.err" || exit $?
timeout -k 10 300 python3 -u bench.py --only-leg dataset_splits > "$OUT/splits.json" 2> "$OUT/splits.err" || exit $?
echo done
