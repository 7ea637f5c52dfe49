#!/usr/bin/env bash
# Fused stream + projection kernel: parity tests, then the in-process A/B.
set -u
TAG=${1:-fused}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mmb2.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "stream_project" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
[ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 300 python3 -u tools/fused_ab.py ${AB_ARGS:-} > "$OUT/ab.txt" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.txt"
exit $rc
