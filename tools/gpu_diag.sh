#!/usr/bin/env bash
# GPU tests (optional: SKIP_TESTS=1), then the projection ablation (tools/proj_diag.py).
set -u
OUT=$PWD/gpurun_out/${TAG:-diag}; mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
fi
timeout -k 10 400 python3 -u tools/proj_diag.py "$@" > "$OUT/diag.log" 2>&1
rc=$?; cat "$OUT/diag.log" | tail -12; exit $rc
